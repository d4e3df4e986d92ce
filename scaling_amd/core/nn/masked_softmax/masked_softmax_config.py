from enum import Enum

from pydantic import Field

from ...config import BaseConfig


class MaskedSoftmaxKernel(Enum):
    TORCH = "torch"
    FLASH_ATTENTION = "flash_attention"


class MaskedSoftmaxConfig(BaseConfig):
    kernel: MaskedSoftmaxKernel = Field(
        MaskedSoftmaxKernel.TORCH,
        description="'flash_attention' selects the MI355X HIP flash-attention kernel; 'torch' the unfused "
        "masked-softmax path (needed for attention score manipulation)",
    )
    softmax_in_fp32: bool = Field(False, description="Cast scores to fp32 before the softmax")
    scale: float = Field(1.0, description="Scale with which scores are multiplied (not divided!) before softmax")
    deterministic_flash_attn_bwd: bool = Field(
        False,
        description="request a bitwise-reproducible flash-attention backward (the reference's flash-attn flag). "
        "On MI355X the reproducible two-kernel backward (one owner workgroup per dK/dV block and per dQ block) is "
        "also the fastest: a one-pass backward that adds dQ with fp32 atomics is floored by the chip's ~1.3 TB/s "
        "float-atomic rate at 108.7 ms per Llama-2-7B step for the dQ adds alone (profiles/atomic_dq_floor_r3.json) "
        "against 47 ms for the whole deterministic dQ pass, so False (reproducibility not required) selects the "
        "same kernels as True",
    )
