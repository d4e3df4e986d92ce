from .get_norm import NormType, get_norm
from .layernorm import LayerNorm
from .layernorm_config import LayerNormConfig, LayerNormOptimizationType
from .rms_norm import RMSNorm

__all__ = ["LayerNorm", "LayerNormConfig", "LayerNormOptimizationType", "NormType", "RMSNorm", "get_norm"]
