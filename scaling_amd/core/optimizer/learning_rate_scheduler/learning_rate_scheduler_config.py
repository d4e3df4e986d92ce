from enum import Enum

from pydantic import Field

from ...config import BaseConfig


class LearningRateDecayStyle(Enum):
    CONSTANT = "constant"
    LINEAR = "linear"
    COSINE = "cosine"


class LearningRateSchedulerConfig(BaseConfig):
    learning_rate: float = Field(0.0, description="Base (= maximum) learning rate.")
    learning_rate_minimum: float = Field(0.0, description="Final learning rate after decay.")
    learning_rate_decay_style: LearningRateDecayStyle = Field(
        LearningRateDecayStyle.COSINE, description="Shape of the learning rate decay after warm up"
    )
    learning_rate_decay_iters: int = Field(0, description="Iterations of the schedule (warmup included).")
    learning_rate_warmup_steps: int = Field(0, description="Linear warmup steps.")
