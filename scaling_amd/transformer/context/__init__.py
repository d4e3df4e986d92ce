from .config import (
    AdapterConfig,
    BitfitBiasConfig,
    DataConfig,
    EmbeddingHeadConfig,
    MLPType,
    Precision,
    SoftpromptConfig,
    TrainingConfig,
    TransformerArchitectureConfig,
    TransformerConfig,
)
from .context import TransformerContext
from ...core import LearningRateSchedulerConfig, OptimizerConfig

__all__ = [
    "AdapterConfig",
    "BitfitBiasConfig",
    "DataConfig",
    "EmbeddingHeadConfig",
    "LearningRateSchedulerConfig",
    "OptimizerConfig",
    "MLPType",
    "Precision",
    "SoftpromptConfig",
    "TrainingConfig",
    "TransformerArchitectureConfig",
    "TransformerConfig",
    "TransformerContext",
]
