"""Unfused masked softmax (reference ``masked_softmax.py:8-50``): optional fp32 upcast, multiply by
``scale``, fill masked positions with -10000, softmax over the last dim."""
from __future__ import annotations

from typing import Optional

import torch

from .masked_softmax_config import MaskedSoftmaxConfig, MaskedSoftmaxKernel


class MaskedSoftmaxTorch(torch.nn.Module):
    def __init__(self, config: MaskedSoftmaxConfig) -> None:
        super().__init__()
        self.config = config

    def forward(self, x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        in_dtype = x.dtype
        if self.config.softmax_in_fp32 and x.dtype != torch.float32:
            x = x.float()
        if self.config.scale != 1.0:
            x = x * self.config.scale
        x = x.masked_fill(mask.to(x.device), -10000.0)
        probs = torch.softmax(x, dim=-1)
        return probs.to(in_dtype) if self.config.softmax_in_fp32 else probs


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
