from .activation_function import ActivationFunction, get_activation_function
from .attention import ParallelSelfAttention, RelativePositionEmbeddingType
from .linear import ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding
from .lora import ParallelLoRa
from .lora_config import LoRaConfig, LoRAModuleType
from .masked_softmax import MaskedSoftmax, MaskedSoftmaxConfig, MaskedSoftmaxKernel
from .mlp import ParallelMLP, ParallelSwiGLUMLP
from .norm import LayerNorm, LayerNormConfig, LayerNormOptimizationType, NormType, RMSNorm, get_norm
from .parallel_module import (
    BaseLayer,
    InferenceModule,
    LayerSpec,
    ParallelModule,
    PipePartitionCoordinates,
    TiedLayerSpec,
    pipe_partition_uniform,
)
from .parameter_meta import CoreParameterMeta
from .pipeline_schedule import PipelineScheduleInference, PipelineScheduleTrain
from .rotary import RotaryEmbedding, RotaryEmbeddingComplex
from .rotary_config import RotaryConfig

__all__ = [
    "ActivationFunction",
    "BaseLayer",
    "ColumnParallelLinear",
    "CoreParameterMeta",
    "InferenceModule",
    "LayerNorm",
    "LayerNormConfig",
    "LayerNormOptimizationType",
    "LayerSpec",
    "LoRAModuleType",
    "LoRaConfig",
    "MaskedSoftmax",
    "MaskedSoftmaxConfig",
    "MaskedSoftmaxKernel",
    "NormType",
    "ParallelLoRa",
    "ParallelMLP",
    "ParallelModule",
    "ParallelSelfAttention",
    "ParallelSwiGLUMLP",
    "PipePartitionCoordinates",
    "PipelineScheduleInference",
    "PipelineScheduleTrain",
    "RMSNorm",
    "RelativePositionEmbeddingType",
    "RotaryConfig",
    "RotaryEmbedding",
    "RotaryEmbeddingComplex",
    "RowParallelLinear",
    "TiedLayerSpec",
    "VocabParallelEmbedding",
    "get_activation_function",
    "get_norm",
    "pipe_partition_uniform",
]
