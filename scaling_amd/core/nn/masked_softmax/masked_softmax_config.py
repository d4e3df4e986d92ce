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
        False, description="kept for config compatibility: the HIP flash backward is always deterministic"
    )
