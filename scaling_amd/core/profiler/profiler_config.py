from pathlib import Path
from typing import Optional

from pydantic import Field

from ..config import BaseConfig


class ProfilerConfig(BaseConfig):
    """Instruction-level profiler (reference ``src/scaling/core/profiler/profiler_config.py:9``)."""

    profile_steps: int = Field(0, description="number of to be timed steps, will not run profiling if set to 0")
    profile_start_at_step: int = Field(10, description="start profiling after this many steps")
    profiler_output: Optional[Path] = Field(None, description="output json file of the profiler")
    use_events: bool = Field(
        True,
        description="MI355X: time instructions with HIP events on the compute stream instead of "
        "device-wide synchronizes (set False for the reference's synchronizing timers)",
    )
