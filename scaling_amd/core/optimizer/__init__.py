from .allreduce import allreduce_no_retain, allreduce_tensor_in_float32
from .base import BaseOptimizer, BaseOptimizerState, OptimizerStepOutput
from .learning_rate_scheduler import LearningRateDecayStyle, LearningRateScheduler, LearningRateSchedulerConfig
from .loss_scaler import LossScaler
from .loss_scaler_config import LossScalerConfig
from .optimizer import Optimizer
from .optimizer_config import OptimizerConfig
from .parameter_group import OptimizerParamGroup
from .parameter_group_config import OptimizerParamGroupConfig

__all__ = [
    "BaseOptimizer",
    "BaseOptimizerState",
    "LearningRateDecayStyle",
    "LearningRateScheduler",
    "LearningRateSchedulerConfig",
    "LossScaler",
    "LossScalerConfig",
    "Optimizer",
    "OptimizerConfig",
    "OptimizerParamGroup",
    "OptimizerParamGroupConfig",
    "OptimizerStepOutput",
    "allreduce_no_retain",
    "allreduce_tensor_in_float32",
]
