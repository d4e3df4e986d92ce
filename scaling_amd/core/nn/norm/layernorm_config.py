from enum import Enum

from pydantic import Field

from ...config import BaseConfig


class LayerNormOptimizationType(Enum):
    TORCH = "torch"
    # MI355X-native fused HIP kernel (default on GPU regardless of this flag; kept for config parity)
    FUSED = "fused"


class LayerNormConfig(BaseConfig):
    optimization_type: LayerNormOptimizationType = Field(
        LayerNormOptimizationType.TORCH, description="kept for config compatibility; GPU always uses the HIP kernel"
    )
    layernorm_epsilon: float = Field(1.0e-5, description="A value added to the denominator for numerical stability")
