"""SwiGLU ``silu(a) * b`` with a fused HIP forward/backward (``csrc/kernels/swiglu_rope.hip``).

``swiglu_fused(z)`` takes the output of ONE fused ``[dense_in ; siglu_weight]`` GEMM (``[..., 2F]``)
and returns ``[..., F]``; its backward writes the fused ``[..., 2F]`` gradient directly, so the
backward of the fused GEMM needs no concatenation.
"""
from __future__ import annotations

from typing import Any

import torch

from ._ext import ext, use_native


class _SwiGLUFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, z: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        F = z.shape[-1] // 2
        zc = z.contiguous()
        a, b = zc[..., :F], zc[..., F:]
        ctx.save_for_backward(zc)
        return ext().swiglu_fwd(a, b)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> tuple:  # type: ignore[override]
        (z,) = ctx.saved_tensors
        F = z.shape[-1] // 2
        (dz,) = ext().swiglu_bwd(dy, z[..., :F], z[..., F:], True)
        return (dz,)


class _SwiGLU2(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        a, b = a.contiguous(), b.contiguous()
        ctx.save_for_backward(a, b)
        return ext().swiglu_fwd(a, b)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> tuple:  # type: ignore[override]
        a, b = ctx.saved_tensors
        da, db = ext().swiglu_bwd(dy, a, b, False)
        return da, db


def swiglu_reference(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return torch.nn.functional.silu(a) * b


def swiglu(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if use_native(a) and a.shape[-1] % 8 == 0:
        return _SwiGLU2.apply(a, b)
    return swiglu_reference(a, b)


def swiglu_fused(z: torch.Tensor) -> torch.Tensor:
    F = z.shape[-1] // 2
    if use_native(z) and F % 8 == 0:
        return _SwiGLUFused.apply(z)
    return swiglu_reference(z[..., :F], z[..., F:])
