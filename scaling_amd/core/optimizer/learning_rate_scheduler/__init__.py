from .learning_rate_scheduler import LearningRateScheduler
from .learning_rate_scheduler_config import LearningRateDecayStyle, LearningRateSchedulerConfig

__all__ = ["LearningRateDecayStyle", "LearningRateScheduler", "LearningRateSchedulerConfig"]
