"""RMSNorm / LayerNorm with fused HIP forward/backward (``csrc/kernels/norm.hip``)."""
from __future__ import annotations

from typing import Any, Optional

import torch

from ._ext import ext, use_native


def rms_norm_reference(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    # reference numerics: (x * rsqrt(mean(x^2) + eps)).type_as(x) * w   (rms_norm.py:45-56)
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).type_as(x) * w


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:  # type: ignore[override]
        xc = x.contiguous()
        y, _, rstd = ext().norm_fwd(xc, w.contiguous(), None, eps, False)
        ctx.save_for_backward(xc, w, rstd)
        return y

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> tuple:  # type: ignore[override]
        x, w, rstd = ctx.saved_tensors
        empty = rstd.new_empty(0)
        dx, dw, _ = ext().norm_bwd(dy.contiguous(), x, w.contiguous(), empty, rstd, False)
        return dx, dw, None


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:  # type: ignore[override]
        xc = x.contiguous()
        y, mean, rstd = ext().norm_fwd(xc, w.contiguous(), b.contiguous(), eps, True)
        ctx.save_for_backward(xc, w, mean, rstd)
        return y

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> tuple:  # type: ignore[override]
        x, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = ext().norm_bwd(dy.contiguous(), x, w.contiguous(), mean, rstd, True)
        return dx, dw, db, None


def _native_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return use_native(x) and x.dtype == w.dtype and x.shape[-1] % 8 == 0


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    if _native_ok(x, w):
        return _RMSNorm.apply(x, w, eps)
    if use_native(x):
        raise RuntimeError(f"rms_norm: unsupported GPU input (dtype {x.dtype}/{w.dtype}, hidden {x.shape[-1]})")
    return rms_norm_reference(x, w, eps)


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], eps: float) -> torch.Tensor:
    if b is not None and _native_ok(x, w) and b.dtype == w.dtype:
        return _LayerNorm.apply(x, w, b, eps)
    if use_native(x) and b is not None:
        raise RuntimeError(f"layer_norm: unsupported GPU input (dtype {x.dtype}/{w.dtype}, hidden {x.shape[-1]})")
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)
