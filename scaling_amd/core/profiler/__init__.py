from .profiler import Profiler, ProfilerObservation
from .profiler_config import ProfilerConfig
from .timer import EventTimer, SynchronizedTimer

__all__ = ["EventTimer", "Profiler", "ProfilerConfig", "ProfilerObservation", "SynchronizedTimer"]
