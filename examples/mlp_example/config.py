"""Config tree of the MLP example (reference ``examples/mlp_example/config.py``)."""
from pydantic import Field

from scaling_amd.core import (
    BaseConfig,
    LearningRateSchedulerConfig,
    OptimizerConfig,
    ProfilerConfig,
    RunnerConfig,
    TopologyConfig,
    TrainerConfig,
)
from scaling_amd.core.logging import LoggerConfig


class MLPArchitectureConfig(BaseConfig):
    n_hidden_layers: int = Field(0, ge=0, description="Hidden layers between the input and output layers.")
    hidden_dim: int = Field(64, gt=0, description="Units per hidden layer.")


class TrainingConfig(BaseConfig):
    weight_decay: float = Field(0.0001, description="")


class DataConfig(BaseConfig):
    mnist_root: str = Field(".data", description="directory holding the MNIST idx files (synthetic data when absent)")
    synthetic_samples: int = Field(8192, description="size of the synthetic train set used without MNIST files")


class MLPConfig(BaseConfig):
    runner: RunnerConfig = Field(RunnerConfig(), description="")
    logger: LoggerConfig = Field(LoggerConfig(), description="")
    topology: TopologyConfig = Field(
        TopologyConfig(model_parallel_size=1, pipe_parallel_size=1, data_parallel_size=1, micro_batch_size=2,  # type: ignore[call-arg]
                       gradient_accumulation_steps=1),
        description="",
    )
    optimizer: OptimizerConfig = Field(OptimizerConfig(), description="")
    learning_rate_scheduler: LearningRateSchedulerConfig = Field(LearningRateSchedulerConfig(), description="")
    training: TrainingConfig = Field(TrainingConfig(), description="")
    trainer: TrainerConfig = Field(TrainerConfig(), description="")
    profiler: ProfilerConfig = Field(ProfilerConfig(), description="")
    architecture: MLPArchitectureConfig = Field(MLPArchitectureConfig(), description="")
    data: DataConfig = Field(DataConfig(), description="")
