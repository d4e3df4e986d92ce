"""RMSNorm / LayerNorm with fused HIP forward/backward (``csrc/kernels/norm.hip``).

``add_rms_norm`` / ``add_layer_norm`` fuse the residual add in front of the norm: the forward reads
``x`` and ``res`` once and writes both ``s = x + res`` and ``norm(s)``; the backward adds the gradient
arriving at ``s`` through the residual stream into the norm's input gradient in the same pass.
"""
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
        y, _, rstd, _ = ext().norm_fwd(xc, w.contiguous(), None, eps, False)
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
        y, mean, rstd, _ = ext().norm_fwd(xc, w.contiguous(), b.contiguous(), eps, True)
        ctx.save_for_backward(xc, w, mean, rstd)
        return y

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> tuple:  # type: ignore[override]
        x, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = ext().norm_bwd(dy.contiguous(), x, w.contiguous(), mean, rstd, True)
        return dx, dw, db, None


class _AddNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, res: Optional[torch.Tensor], w: torch.Tensor, b: Optional[torch.Tensor],
                eps: float, layer: bool) -> tuple:  # type: ignore[override]
        xc = x.contiguous()
        y, mean, rstd, s = ext().norm_fwd(xc, w.contiguous(), None if b is None else b.contiguous(), eps, layer,
                                          None if res is None else res.contiguous())
        if res is None:  # pass-through: s is x itself, its gradient is folded into the norm backward
            s = xc.view_as(xc) if xc is x else xc
        ctx.save_for_backward(s, w, mean, rstd)
        ctx.has_res = res is not None
        ctx.layer = layer
        return s, y

    @staticmethod
    def backward(ctx: Any, ds: Optional[torch.Tensor], dy: Optional[torch.Tensor]) -> tuple:  # type: ignore[override]
        s, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            dx = ds
            dw = torch.zeros_like(w)
            db = torch.zeros_like(w) if ctx.layer else None
        else:
            dx, dw, db = ext().norm_bwd(dy.contiguous(), s, w.contiguous(), mean, rstd, ctx.layer,
                                        None if ds is None else ds.contiguous())
            if not ctx.layer:
                db = None
        return dx, dx if ctx.has_res else None, dw, db, None, None


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


def _res_ok(x: torch.Tensor, res: Optional[torch.Tensor]) -> bool:
    return res is None or (res.shape == x.shape and res.dtype == x.dtype)


def add_rms_norm(x: torch.Tensor, res: Optional[torch.Tensor], w: torch.Tensor, eps: float
                 ) -> tuple[torch.Tensor, torch.Tensor]:
    """``s = x + res; return s, rms_norm(s)`` with the add fused into the norm kernels.

    ``res=None`` returns ``(x, rms_norm(x))``: the residual branch's gradient is then added to the norm's input
    gradient inside the backward kernel instead of by a separate accumulation pass."""
    if _native_ok(x, w) and _res_ok(x, res):
        return _AddNorm.apply(x, res, w, None, eps, False)
    if use_native(x):
        raise RuntimeError(f"add_rms_norm: unsupported GPU input (dtype {x.dtype}/{w.dtype}, shape {x.shape})")
    s = x if res is None else x + res
    return s, rms_norm_reference(s, w, eps)


def add_layer_norm(x: torch.Tensor, res: Optional[torch.Tensor], w: torch.Tensor, b: torch.Tensor, eps: float
                   ) -> tuple[torch.Tensor, torch.Tensor]:
    """``s = x + res; return s, layer_norm(s)`` with the add fused into the norm kernels (``res=None``: pass-through)."""
    if _native_ok(x, w) and b.dtype == w.dtype and _res_ok(x, res):
        return _AddNorm.apply(x, res, w, b, eps, True)
    if use_native(x):
        raise RuntimeError(f"add_layer_norm: unsupported GPU input (dtype {x.dtype}/{w.dtype}, shape {x.shape})")
    s = x if res is None else x + res
    return s, torch.nn.functional.layer_norm(s, (s.shape[-1],), w, b, eps)
