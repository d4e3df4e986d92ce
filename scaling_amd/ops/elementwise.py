"""Masked softmax, activations and dropout(+residual) on the gfx950 kernels of ``csrc/kernels/elementwise.hip``.

* :func:`masked_softmax` — the reference's unfused attention softmax (``masked_softmax.py:14-30``):
  ``softmax(masked_fill(x * scale, mask, -10000))`` over the last dim with fp32 math; when the softmax is
  not forced to fp32, ``x * scale`` and the fill value are rounded through the input dtype exactly as
  torch does on half tensors.
* :func:`activation` — GELU (erf or tanh) / SiLU fwd+bwd (reference ``nn/activation_function.py``).
* :func:`dropout_add` — ``residual + dropout(x)`` in one pass (reference ``layer.py:211-233``); the keep
  mask is a hash of (seed, element index) regenerated in the backward, so no mask tensor is stored.  The
  seed comes from the device generator (:func:`scaling_amd.ops.attention.dropout_seed`), so the TP-constant
  RNG tracker and activation-checkpoint recompute reproduce the same mask.
CPU tensors run the PyTorch reference math.
"""
from __future__ import annotations

from typing import Any, Optional

import torch

from ._ext import ext, use_native
from .attention import dropout_seed

ACT_KINDS = {"gelu": 0, "silu": 1, "gelu_tanh": 2}


def masked_softmax_reference(x: torch.Tensor, mask: Optional[torch.Tensor], scale: float,
                             softmax_in_fp32: bool) -> torch.Tensor:
    in_dtype = x.dtype
    if softmax_in_fp32 and x.dtype != torch.float32:
        x = x.float()
    if scale != 1.0:
        x = x * scale
    if mask is not None:
        x = x.masked_fill(mask.to(x.device), -10000.0)
    probs = torch.softmax(x, dim=-1)
    return probs.to(in_dtype)


class _MaskedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, mask: Optional[torch.Tensor], scale: float, round_scaled: bool):  # type: ignore[override]
        fill = -10000.0
        if round_scaled:
            fill = float(torch.tensor(fill, dtype=x.dtype).item())
        y = ext().masked_softmax_fwd(x, mask, scale, fill, round_scaled)
        ctx.save_for_backward(y, mask if mask is not None else torch.empty(0))
        ctx.has_mask = mask is not None
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor):  # type: ignore[override]
        y, mask = ctx.saved_tensors
        dx = ext().masked_softmax_bwd(dy.contiguous(), y, mask if ctx.has_mask else None, ctx.scale)
        return dx, None, None, None


def masked_softmax(x: torch.Tensor, mask: Optional[torch.Tensor], scale: float = 1.0,
                   softmax_in_fp32: bool = False) -> torch.Tensor:
    """x: [B, H, Sq, Sk]; mask: bool broadcastable to x (True = masked).  Output has x's dtype."""
    if use_native(x) and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16, torch.float16):
        round_scaled = (not softmax_in_fp32) and x.dtype != torch.float32
        return _MaskedSoftmax.apply(x, mask, float(scale), round_scaled)
    return masked_softmax_reference(x, mask, scale, softmax_in_fp32)


class _Activation(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, kind: int):  # type: ignore[override]
        ctx.save_for_backward(x)
        ctx.kind = kind
        return ext().act_fwd(x, kind)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor):  # type: ignore[override]
        (x,) = ctx.saved_tensors
        return ext().act_bwd(dy.contiguous(), x, ctx.kind), None


def activation(x: torch.Tensor, kind: str = "gelu") -> torch.Tensor:
    if use_native(x) and x.dtype in (torch.float32, torch.bfloat16, torch.float16):
        return _Activation.apply(x, ACT_KINDS[kind])
    if kind == "silu":
        return torch.nn.functional.silu(x)
    return torch.nn.functional.gelu(x, approximate="tanh" if kind == "gelu_tanh" else "none")


class _DropoutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, res: Optional[torch.Tensor], p: float, seed: int):  # type: ignore[override]
        ctx.p, ctx.seed, ctx.has_res = p, seed, res is not None
        return ext().dropout_add(x, res, p, seed)

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        dx = ext().dropout_add(g.contiguous(), None, ctx.p, ctx.seed)
        return dx, (g if ctx.has_res else None), None, None


def dropout_add(x: torch.Tensor, residual: Optional[torch.Tensor], p: float, training: bool = True) -> torch.Tensor:
    """``residual + dropout(x, p)`` (``residual`` None: plain dropout)."""
    if p == 0.0 or not training:
        return x if residual is None else residual + x
    if use_native(x) and x.dtype in (torch.float32, torch.bfloat16, torch.float16) and (
            residual is None or residual.dtype == x.dtype):
        return _DropoutAdd.apply(x, residual, float(p), dropout_seed(x.device))
    d = torch.nn.functional.dropout(x, p, training=True)
    return d if residual is None else residual + d
