"""Weight-gradient GEMM ``dW (+)= dY^T X`` on the hand-written gfx950 kernel (``csrc/kernels/gemm.hip``).

Both operands arrive token-major (``dY: [T, N]``, ``X: [T, K]``), i.e. k-strided for this product; the
kernel stages them as they lie (LDS-DMA) and builds MFMA fragments with the transposing LDS read, in a
ping-pong schedule.  At the 7B layer shapes it runs 1.05-1.25 PF vs hipBLASLt's 0.95-1.2 PF
(``profiles/gemm_wgrad_r1.log``).  Shapes it does not tile (M/N not multiples of 256, T not a multiple
of 64) use ``torch.matmul`` / ``addmm_`` (hipBLASLt).

``linear`` is the forward ``x W^T (+ b)`` of every linear layer: at most 4 token rows (token-by-token decoding)
run the weight-streaming GEMV kernel (``csrc/kernels/gemv.hip``), everything else hipBLASLt.
"""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import ext, use_native


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """``out (+)= dy^T @ x`` for 2-D ``dy [T, N]``, ``x [T, K]``; returns ``out`` ([N, K])."""
    if use_native(dy):
        o = out if out is not None else torch.empty(dy.shape[1], x.shape[1], device=dy.device, dtype=dy.dtype)
        if ext().gemm_tn_ok(dy, x, o):
            ext().gemm_tn(dy, x, o, bool(accumulate and out is not None))
            return o
    if out is None:
        return torch.matmul(dy.t(), x)
    if accumulate:
        return out.addmm_(dy.t(), x)
    return torch.matmul(dy.t(), x, out=out)


def transpose2d(x: torch.Tensor) -> torch.Tensor:
    """Contiguous ``x^T`` of a 2-D matrix (LDS-tiled HIP kernel for bf16/fp16 at multiples of 64)."""
    if use_native(x) and ext().transpose_ok(x):
        return ext().transpose2d(x)
    return x.t().contiguous()


GEMV_MAX_ROWS = 4


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.linear(x, w, b)``; decode-sized inputs (<= 4 rows) on the GEMV kernel.

    The GEMV kernel is a raw op without autograd, so it only serves calls that build no graph (grad mode off, or
    no operand requiring grad); a tiny training micro-batch through a tied head keeps ``F.linear``'s backward."""
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    needs_graph = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or (b is not None and b.requires_grad))
    if 0 < rows <= GEMV_MAX_ROWS and not needs_graph and use_native(x) and w.dim() == 2:
        x2 = x.reshape(rows, K)
        if ext().gemv_ok(x2, w) and (b is None or b.dtype == w.dtype):
            return ext().gemv(x2, w, b).reshape(*x.shape[:-1], w.shape[0])
    return torch.nn.functional.linear(x, w, b)
