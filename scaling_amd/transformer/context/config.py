"""Transformer training configuration (schema-compatible with reference
``src/scaling/transformer/context/config.py:28-459``: same sections, field names, defaults and the
``from_dict`` auto-fill of ``trainer.separate_file_for_parameters`` for bitfit/adapter/softprompt)."""
from __future__ import annotations

from copy import deepcopy
from enum import Enum
from pathlib import Path
from typing import Any, Mapping, Optional

import torch
from pydantic import Field, model_validator

from ...core import (
    BaseConfig,
    BlendedDatasetConfig,
    LayerNormConfig,
    LearningRateSchedulerConfig,
    LoRaConfig,
    MaskedSoftmaxConfig,
    NormType,
    OptimizerConfig,
    ProfilerConfig,
    RelativePositionEmbeddingType,
    RunnerConfig,
    TopologyConfig,
    TrainerConfig,
)
from ...core.logging import LoggerConfig

_VERSION_DOC = "model version reported by inference stacks (alpha-numerically increasing)"


class Precision(Enum):
    FLOAT16 = "float16"
    BFLOAT16 = "bfloat16"
    FLOAT32 = "float32"

    @property
    def dtype(self) -> torch.dtype:
        return {"float16": torch.float16, "bfloat16": torch.bfloat16, "float32": torch.float32}[self.value]


class MLPType(Enum):
    DEFAULT = "default"
    SWIGLU = "swiglu"


class TrainingConfig(BaseConfig, populate_by_name=True):
    weight_decay: float = Field(0.0001, description="")
    finetune: bool = Field(False, description="activate finetuning mode")
    finetunable_parameters: list[str] = Field([], description="pattern of parameters to be included in finetuning")
    parameters_exclude: list[str] = Field([], description="pattern of parameters to be excluded in training")
    use_separate_lr_on_embeddings: bool = Field(False, description="", alias="use_seperate_lr_on_embeddings")
    use_deterministic_torch_algorithms: bool = Field(False, description="deterministic torch/hipBLASLt algorithms")

    @model_validator(mode="after")
    def check_finetune(self) -> "TrainingConfig":
        if self.finetune != bool(self.finetunable_parameters):
            raise ValueError(
                "Can not set finetune when finetunable_parameters is empty"
                if self.finetune
                else "Can not set finetunable_parameters when finetune is False"
            )
        return self


class BitfitBiasConfig(BaseConfig):
    name: str = Field(description="")
    version: str = Field(default=".unknown.", description=_VERSION_DOC)


class SoftpromptConfig(BaseConfig):
    name: str = Field(description="")
    n_tokens: int = Field(description="")
    version: str = Field(default=".unknown.", description=_VERSION_DOC)


class AdapterConfig(BaseConfig):
    name: str = Field(description="")
    attention_downsampling_factor: Optional[float] = Field(None, description="")
    mlp_downsampling_factor: Optional[float] = Field(None, description="")
    init_std: float = Field(1.0e-5, description="")
    version: str = Field(default=".unknown.", description=_VERSION_DOC)


class EmbeddingHeadConfig(BaseConfig):
    name: str = Field(description="")
    proj_layers: list[int] = Field(description="")


class TransformerArchitectureConfig(BaseConfig):
    """Constant architecture description of the transformer."""

    vocab_size: int = Field(0, description="tokenizer vocabulary size")
    vocab_file: Optional[Path] = Field(None, description="")
    hidden_size: int = Field(0, description="Transformer hidden size.")
    num_layers: int = Field(0, description="Number of transformer layers")
    num_attention_heads: int = Field(0, description="Number of attention heads")
    num_local_attention_heads: int = Field(0, description="Number of sliding-window attention heads")
    local_attention_window_size: Optional[int] = Field(None, description="The size of the local attention window")
    rotary_embedding_base: int = Field(10000, description="")
    rotary_percentage: float = Field(1.0, description="fraction of each head's dims that get rotary embeddings")
    sequence_length: int = Field(2048, description="tokens per sample")
    norm_type: NormType = Field(NormType.LAYERNORM, description="'layernorm' or 'rms'")
    relative_position_embedding_type: RelativePositionEmbeddingType = Field(
        RelativePositionEmbeddingType.ROTARY, description="'none', 'rotary', 'rotary_complex'"
    )
    mlp_type: MLPType = Field(MLPType.DEFAULT, description="'default' or 'swiglu'")
    mlp_factor: float = Field(4.0, description="expansion factor for mlp hidden layer")
    attention_bias: bool = Field(True, description="add bias terms to attention components")
    attention_qkv_in_one: bool = Field(True, description="query/key/value as one fused projection")
    attention_num_kv_heads: Optional[int] = Field(None, description="number kv heads, if it differs from query heads")
    attention_use_matmul: bool = Field(False, description="use torch.matmul instead of torch.baddbmm")
    mlp_bias: bool = Field(True, description="add bias terms to mlp")
    key_query_norm: bool = Field(False, description="add a norm for key and query scores")
    weight_tying: bool = Field(True, description="")
    masked_softmax: MaskedSoftmaxConfig = Field(MaskedSoftmaxConfig(), description="")
    layernorm: LayerNormConfig = Field(LayerNormConfig(), description="")
    precision: Precision = Field(Precision.FLOAT32, description="")
    dropout_embedding: float = Field(0.0, description="", ge=0.0, le=1.0)
    dropout_attention_probs: float = Field(0.0, description="", ge=0.0, le=1.0)
    dropout_after_attention: float = Field(0.0, description="", ge=0.0, le=1.0)
    dropout_after_mlp: float = Field(0.0, description="", ge=0.0, le=1.0)
    bitfit_bias_config: Optional[BitfitBiasConfig] = Field(None, description="Config for a bias that will be finetuned.")
    finetunable_token_ids: list[int] = Field(list(), description="embedding rows that stay trainable in finetuning")
    image_encoder: bool = Field(False, description="add image encoder to input embedding")
    dropout_image_encoder: float = Field(0.0, description="", ge=0.0, le=1.0)
    softprompt_config: Optional[SoftpromptConfig] = Field(None, description="")
    adapter_config: Optional[AdapterConfig] = Field(None, description="")
    lora_config: Optional[LoRaConfig] = Field(None, description="creates LoRa finetuning configuration")
    embedding_head_config: Optional[EmbeddingHeadConfig] = Field(None, description="")
    causal: bool = Field(True, description="Make attention layers causal.")


class DataConfig(BaseConfig):
    """Dataset configuration."""

    legacy_dataset: bool = Field(False, description="Use the legacy (Megatron MMIDIDX) dataset implementation")
    load_mmap_index_to_memory: bool = Field(False, description="")
    use_mmap: bool = Field(True, description="Use memory maps instead of regular file operations to read data")
    load_data_item_mmap_index_to_memory: bool = Field(False, description="")
    finetuning_dataset: bool = Field(False, description="Use the finetuning text dataset implementation")
    finetuning_chat_dataset: bool = Field(False, description="Use the finetuning chat dataset implementation")
    finetuning_dataset_memory_map: bool = Field(False, description="finetuning dataset is a memory map")
    data_prefixes: Optional[list[Path]] = Field(None, description="Training data prefixes")
    validation_data_prefixes: Optional[list[Path]] = Field(None, description="Validation data prefixes")
    blended_dataset: BlendedDatasetConfig = Field(BlendedDatasetConfig(), description="")
    only_full_sequences: bool = Field(False, description="only use sequences that fully fill the context")
    allow_incomplete_sequences_every_n: int = Field(0, description="with only_full_sequences: every n-th may be partial")


class TransformerConfig(BaseConfig):
    version: str = Field(default=".unknown.", description=_VERSION_DOC)
    runner: RunnerConfig = Field(RunnerConfig(), description="")
    logger: LoggerConfig = Field(LoggerConfig(), description="")
    topology: TopologyConfig = Field(
        TopologyConfig(  # type: ignore[call-arg]
            model_parallel_size=1, pipe_parallel_size=1, data_parallel_size=1, micro_batch_size=2,
            gradient_accumulation_steps=1,
        ),
        description="",
    )
    optimizer: OptimizerConfig = Field(OptimizerConfig(), description="")
    learning_rate_scheduler: LearningRateSchedulerConfig = Field(LearningRateSchedulerConfig(), description="")
    embedding_learning_rate_scheduler: LearningRateSchedulerConfig = Field(LearningRateSchedulerConfig(), description="")
    training: TrainingConfig = Field(TrainingConfig(), description="")
    trainer: TrainerConfig = Field(TrainerConfig(), description="")
    profiler: ProfilerConfig = Field(ProfilerConfig(), description="")
    transformer_architecture: TransformerArchitectureConfig = Field(TransformerArchitectureConfig(), description="")
    data: DataConfig = Field(DataConfig(), description="")
    determined_experiment_id: Optional[int] = Field(None, description="")
    determined_trial_id: Optional[int] = Field(None, description="")

    @classmethod
    def from_dict(cls, d: Mapping[str, Any], overwrite_values: Optional[dict] = None) -> "TransformerConfig":  # type: ignore[override]
        arch = d.get("transformer_architecture") or {}
        sep = set()
        for key, prefix in (("bitfit_bias_config", "bias"), ("adapter_config", "adapter"), ("softprompt_config", "softprompt")):
            if arch.get(key) is not None:
                sep.add(f"{prefix}_{arch[key]['name']}")
        d2 = dict(deepcopy(d))
        if sep:
            d2.setdefault("trainer", {})
            d2["trainer"] = dict(d2["trainer"] or {})
            d2["trainer"]["separate_file_for_parameters"] = sorted(sep)
        return super().from_dict(d2, overwrite_values=overwrite_values)
