"""scaling_amd.core — model-agnostic 3D-parallel training engine (API of reference ``scaling.core``)."""
from .config import BaseConfig
from .context import BaseContext, BaseContextGeneric, DeterminedBaseContext
from .data import (
    BaseBlendedDataset,
    BaseDataset,
    BaseDatasetBatch,
    BaseDatasetItem,
    BaseLayerIO,
    BlendedDatasetConfig,
    DataLoader,
    FileDataset,
    MemoryMapDataset,
    MemoryMapDatasetBuilder,
    broadcast_data,
)
from .logging import LoggerConfig, logger
from .nn import (
    ActivationFunction,
    BaseLayer,
    ColumnParallelLinear,
    CoreParameterMeta,
    InferenceModule,
    LayerNorm,
    LayerNormConfig,
    LayerNormOptimizationType,
    LayerSpec,
    LoRaConfig,
    LoRAModuleType,
    MaskedSoftmax,
    MaskedSoftmaxConfig,
    MaskedSoftmaxKernel,
    NormType,
    ParallelLoRa,
    ParallelMLP,
    ParallelModule,
    ParallelSelfAttention,
    ParallelSwiGLUMLP,
    PipelineScheduleInference,
    PipelineScheduleTrain,
    PipePartitionCoordinates,
    RelativePositionEmbeddingType,
    RMSNorm,
    RotaryConfig,
    RotaryEmbedding,
    RotaryEmbeddingComplex,
    RowParallelLinear,
    TiedLayerSpec,
    VocabParallelEmbedding,
    get_activation_function,
    get_norm,
    pipe_partition_uniform,
)
from .optimizer import (
    BaseOptimizer,
    LearningRateDecayStyle,
    LearningRateScheduler,
    LearningRateSchedulerConfig,
    LossScaler,
    LossScalerConfig,
    Optimizer,
    OptimizerConfig,
    OptimizerParamGroup,
    OptimizerParamGroupConfig,
)
from .profiler import Profiler, ProfilerConfig, SynchronizedTimer
from .runner import LaunchConfig, RunnerConfig, RunnerDockerConfig, RunnerType, runner_main
from .topology import PipePartitionMethod, Topology, TopologyConfig
from .trainer import BaseTrainer, DeterminedBaseTrainer, TrainerConfig
