"""Unfused masked softmax (reference ``masked_softmax.py:8-50``): optional fp32 upcast, multiply by
``scale``, fill masked positions with -10000, softmax over the last dim.  On the GPU this is one HIP
kernel per direction (``csrc/kernels/elementwise.hip``, fp32 math, rounding emulated for half inputs)."""
from __future__ import annotations

from typing import Optional

import torch

from ....ops.elementwise import masked_softmax
from .masked_softmax_config import MaskedSoftmaxConfig, MaskedSoftmaxKernel


class MaskedSoftmaxTorch(torch.nn.Module):
    def __init__(self, config: MaskedSoftmaxConfig) -> None:
        super().__init__()
        self.config = config

    def forward(self, x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        return masked_softmax(x, mask, self.config.scale, self.config.softmax_in_fp32)


class MaskedSoftmax(torch.nn.Module):
    def __init__(self, config: MaskedSoftmaxConfig) -> None:
        super().__init__()
        self.config = config
        self.kernel: Optional[torch.nn.Module] = (
            MaskedSoftmaxTorch(config) if config.kernel == MaskedSoftmaxKernel.TORCH else None
        )

    def forward(self, x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        kernel = self.kernel if self.kernel is not None else MaskedSoftmaxTorch(self.config)
        return kernel(x, mask)
