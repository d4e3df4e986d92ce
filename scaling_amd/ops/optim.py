"""Fused optimizer primitives on flat buffers: AdamW step and L2-norm/non-finite reductions."""
from __future__ import annotations

import math
from typing import Optional

import torch

from ._ext import ext, use_native


def adamw_step_(p: torch.Tensor, grad: torch.Tensor, m: torch.Tensor, v: torch.Tensor, *, lr: float, beta1: float,
                beta2: float, eps: float, weight_decay: float, step: int, grad_scale: float = 1.0,
                param_out: Optional[torch.Tensor] = None) -> None:
    """torch.optim.AdamW semantics on flat fp32 (p, m, v); optionally writes the model-dtype param copy."""
    if use_native(p):
        ext().adamw_(p, grad, m, v, param_out, lr, beta1, beta2, eps, weight_decay, step, grad_scale)
        return
    g = grad.float() * grad_scale
    p.mul_(1 - lr * weight_decay)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if param_out is not None:
        param_out.copy_(p)


def sumsq_nonfinite_(x: torch.Tensor, out: torch.Tensor, scale: float = 1.0, accumulate: bool = True) -> None:
    """out[0] (+)= sum((x*scale)^2) over finite entries, out[1] (+)= #non-finite.  out: fp32 [2] on x.device."""
    if use_native(x):
        ext().sumsq_(x.reshape(-1), out, scale, accumulate)
        return
    xf = x.float().reshape(-1) * scale
    fin = torch.isfinite(xf)
    vals = torch.stack([(xf[fin] ** 2).sum(), (~fin).sum().float()])
    if accumulate:
        out[:2] += vals
    else:
        out[:2] = vals


def cast_scale_(x: torch.Tensor, y: torch.Tensor, scale: float = 1.0) -> None:
    if use_native(x) and x.is_contiguous() and y.is_contiguous():
        ext().cast_scale_(x.reshape(-1), y.reshape(-1), scale)
        return
    y.copy_(x * scale if scale != 1.0 else x)
