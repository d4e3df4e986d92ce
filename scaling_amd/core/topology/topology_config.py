"""3D-parallel layout + batch arithmetic config.

Field names/semantics follow the reference ``TopologyConfig``
(``src/scaling/core/topology/topology_config.py:20-206``): 3 of {mp, pp, dp, world_size} and 2 of
{global_batch_size, micro_batch_size, gradient_accumulation_steps} are required, the rest is inferred
and ``global_batch_size == micro_batch_size * gradient_accumulation_steps * data_parallel_size`` is
enforced.  New optional fields (MI355X-specific) default to behaviour-preserving values.
"""
from __future__ import annotations

from enum import Enum
from typing import Any, Optional

from pydantic import Field, model_validator

from ..config import BaseConfig


class PipePartitionMethod(Enum):
    UNIFORM = "uniform"
    BALANCED = "balanced"


class ActivationCheckpointingType(Enum):
    EVERY_PIPE_STAGE = "every_pipe_stage"
    EVERY_LAYER = "every_layer"
    # MI355X addition: per-layer recompute that keeps each layer's flash-attention output + LSE, so the backward's
    # recompute skips the attention forward (``ops.attention.AttentionStash``)
    EVERY_LAYER_KEEP_ATTENTION = "every_layer_keep_attention"
    # MI355X addition: selective per-layer recompute -- the first forward also keeps every linear layer's GEMM output,
    # so the recompute runs only the cheap element-wise work (norms, RoPE, SwiGLU, residual adds) and rebuilds the
    # autograd graph around the kept outputs (``ops.attention.stash_gemm``)
    EVERY_LAYER_SAVE_MATMULS = "every_layer_save_matmuls"
    DISABLED = "disabled"


def _infer_parallel(mp: Optional[int], pp: Optional[int], dp: Optional[int], ws: Optional[int]) -> tuple:
    if sum(v is not None for v in (mp, pp, dp, ws)) < 3:
        raise AssertionError(
            "At least 3 out of 4 parallelization parameters (model_parallel_size, pipe_parallel_size, "
            "data_parallel_size and world_size) need to be set."
        )
    if ws is None:
        ws = mp * pp * dp  # type: ignore[operator]
    elif mp is None:
        mp = ws // (pp * dp)  # type: ignore[operator]
    elif pp is None:
        pp = ws // (mp * dp)  # type: ignore[operator]
    elif dp is None:
        dp = ws // (mp * pp)
    return mp, pp, dp, ws


def _infer_batch(gbs: Optional[int], mbs: Optional[int], acc: Optional[int], dp: int) -> tuple:
    if sum(v is not None for v in (gbs, mbs, acc)) < 2:
        raise AssertionError(
            "At least 2 out of 3 batch size parameters (global_batch_size, micro_batch_size, "
            "and gradient_accumulation_steps) need to be set."
        )
    if acc is None:
        acc = gbs // (mbs * dp)  # type: ignore[operator]
    if mbs is None:
        mbs = gbs // (acc * dp)  # type: ignore[operator]
    if gbs is None:
        gbs = mbs * acc * dp
    assert gbs == mbs * acc * dp, (
        f"global_batch_size {gbs} does not equal the product of micro_batch_size ({mbs}) "
        f"and gradient_accumulation_steps ({acc}) and data_parallel_size ({dp})."
    )
    return gbs, mbs, acc


class TopologyConfig(BaseConfig):
    global_rank: Optional[int] = Field(None, description="global rank of this process", ge=0)
    world_size: int = Field(description="total number of processes", gt=0)
    local_slot: Optional[int] = Field(None, description="local device index of this process", ge=0)
    model_parallel_size: int = Field(description="tensor parallel degree", gt=0)
    pipe_parallel_size: int = Field(description="pipeline parallel degree", gt=0)
    data_parallel_size: int = Field(description="data parallel degree", gt=0)
    global_batch_size: int = Field(
        description="global train batch size including all gradient accumulation steps", gt=0
    )
    micro_batch_size: int = Field(description="Batch size for one training micro step.", gt=0)
    gradient_accumulation_steps: int = Field(description="Number of gradient accumulation steps.", gt=0)
    pipe_partition_method: PipePartitionMethod = Field(
        PipePartitionMethod.UNIFORM, description="Method to assign layers to pipeline stages"
    )
    pipe_partition_overwrite: Optional[list[int]] = Field(None, description="manually set pipe partitions")
    activation_checkpointing_type: ActivationCheckpointingType = Field(
        ActivationCheckpointingType.DISABLED, description="activation checkpointing granularity"
    )
    sequence_parallel: bool = Field(False, description="Megatron sequence parallelism inside the TP group")
    # --- MI355X-native additions (optional) ---
    backend: Optional[str] = Field(
        None,
        description="torch.distributed backend; None selects 'nccl' (RCCL over xGMI) when a GPU is "
        "present and 'gloo' otherwise; 'fake' = one process playing rank global_rank with stubbed collectives "
        "(the per-rank compute proxy, core/topology/stub_collectives.py)",
    )
    gloo_on_gpu: bool = Field(
        False,
        description="rehearsal mode: backend 'gloo' with the ranks' tensors on GPUs (local slot modulo the "
        "visible devices, so several ranks may share one GPU, which RCCL refuses); exercises the GPU-side "
        "multi-rank paths (streams, events, kernels) on a 1-GPU box",
    )
    tensor_parallel_comm_chunks: int = Field(
        1,
        description="row-parallel outputs (attention dense, MLP dense_out) are computed in this many token chunks "
        "and the TP all-reduce (or sequence-parallel reduce-scatter) of chunk i runs on a communication stream "
        "while chunk i+1 is multiplied; 1 = one GEMM then one collective (the reference's order)",
        ge=1,
        le=16,
    )

    @model_validator(mode="before")
    @classmethod
    def validate_parallelization_and_batch(cls, values: dict[Any, Any]) -> dict[Any, Any]:
        mp, pp, dp, ws = _infer_parallel(
            values.get("model_parallel_size"),
            values.get("pipe_parallel_size"),
            values.get("data_parallel_size"),
            values.get("world_size"),
        )
        gbs, mbs, acc = _infer_batch(
            values.get("global_batch_size"),
            values.get("micro_batch_size"),
            values.get("gradient_accumulation_steps"),
            dp,
        )
        values.update(
            world_size=ws,
            model_parallel_size=mp,
            pipe_parallel_size=pp,
            data_parallel_size=dp,
            global_batch_size=gbs,
            micro_batch_size=mbs,
            gradient_accumulation_steps=acc,
        )
        values.setdefault("global_rank", None)
        return values
