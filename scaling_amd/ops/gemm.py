"""Linear-layer GEMMs on the hand-written gfx950 kernels.

``wgrad``: the weight gradient ``dW (+)= dY^T X`` (``csrc/kernels/gemm.hip``, ``gemm_tn_ring_kernel``).

Both operands arrive token-major (``dY: [T, N]``, ``X: [T, K]``), i.e. k-strided for this product; the kernel stages
them as they lie (LDS-DMA into a four-slot ring of 32-deep k-steps) and builds MFMA fragments with the transposing LDS
read, one wave per SIMD, 256 x 256 tiles, 16x16x32 MFMAs accumulating in AGPRs, a split-K tail for the ragged last
round of tiles.  At the 7B layer shapes it runs 1.43-1.55 PF (MFMA util 0.80-0.81, ``profiles/pmc_step_r4.txt``) where
hipBLASLt runs this TN layout at 0.95-1.2 PF.  M / N need only be multiples of 16: the tensor-parallel shards 5504,
2752 and 16000 run in HIP too (ragged edge tiles, ``SCALING_AMD_WGRAD_RAGGED=0`` sends them to hipBLASLt as before
round 5).  Shapes it does not tile (M/N not multiples of 16, T not a multiple of 128) use ``torch.matmul`` /
``addmm_`` (hipBLASLt).

``linear`` is the forward ``x W^T (+ b)`` of every linear layer, ``mm_nt`` the input gradient ``dY (W^T)^T`` on
the cached transpose and ``mm`` the input gradient ``dY W`` without it: at most 4 token rows (token-by-token decoding)
run the weight-streaming GEMV kernel (``csrc/kernels/gemv.hip``); small products (<= ``SCALING_AMD_LT_SMALL_FLOP``
multiply-adds, 2^33 by default: none of the 7B step's) go through cached hipBLASLt plans (``csrc/blaslt.cpp``); the
rest are plain library GEMMs (hipBLASLt through torch, TunableOp table ``scaling_amd/tuning/gemm_gfx950.csv``).  A hand-written NT GEMM with fused SwiGLU epilogues (rounds 3-5) stayed
1-6 % behind hipBLASLt at every 7B shape and lost in the step even with its epilogues
(``profiles/gemm_nt_round_remap_ab_r5.log``, ``profiles/swiglu_bwd_nt_ab_r5.log``); it was deleted in round 6.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ._ext import ext, use_native


_WGRAD_RAGGED = os.environ.get("SCALING_AMD_WGRAD_RAGGED", "1") != "0"
_WGRAD_HIP = os.environ.get("SCALING_AMD_WGRAD_HIP", "1") != "0"  # 0: every weight gradient on hipBLASLt (A/B, forensics)


def wgrad(dy: torch.Tensor, x: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    """``out (+)= dy^T @ x`` for 2-D ``dy [T, N]``, ``x [T, K]``; returns ``out`` ([N, K])."""
    if use_native(dy) and _WGRAD_HIP:
        o = out if out is not None else torch.empty(dy.shape[1], x.shape[1], device=dy.device, dtype=dy.dtype)
        ragged = dy.shape[1] % 256 != 0 or x.shape[1] % 256 != 0
        if (_WGRAD_RAGGED or not ragged) and ext().gemm_tn_ok(dy, x, o):
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
# products of at most this many multiply-adds go through cached hipBLASLt plans (csrc/blaslt.cpp): torch's path
# re-plans every call (~25-30 us of host time), which only a host-bound small model notices; 0 disables
_LT_SMALL = int(os.environ.get("SCALING_AMD_LT_SMALL_FLOP", str(1 << 33)))


def _lt_ok(a: torch.Tensor, w: torch.Tensor, m: int, n: int, k: int) -> bool:
    # (torch's deterministic mode keeps its own library choice: the plans take hipBLASLt's first heuristic pick)
    return (0 < m * n * k <= _LT_SMALL and a.is_cuda and a.dtype in (torch.bfloat16, torch.float16)
            and a.dtype == w.dtype and not torch.are_deterministic_algorithms_enabled()
            and not torch.cuda.is_current_stream_capturing())  # (a plan made inside a capture would own graph memory)


def mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b`` for ``a`` [..., K] and 2-D ``b`` [K, N] (no autograd graph)."""
    K, N = b.shape
    a2 = a.reshape(-1, K)
    if _lt_ok(a, b, a2.shape[0], N, K):
        y = ext().lt_mm(a2.contiguous(), b.contiguous(), a.new_empty(*a.shape[:-1], N))
        if y is not None:
            return y
    return torch.matmul(a, b)


def mm_nt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b^T`` for 2-D ``a`` [M, K] and ``b`` [N, K] (no autograd graph)."""
    if _lt_ok(a, b, a.shape[0], b.shape[0], a.shape[1]):
        y = ext().lt_linear(a.contiguous(), b.contiguous(), None)
        if y is not None:
            return y
    return torch.matmul(a, b.t())


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
    if not needs_graph and w.dim() == 2 and _lt_ok(x, w, rows, w.shape[0], K) and (b is None or b.dtype == w.dtype):
        # (written into the un-flattened output: a view of a 2-D result would not be updatable in place -- the
        # in-base LoRA up-projections accumulate into the q/k/v GEMM output)
        y = ext().lt_linear(x.reshape(rows, K).contiguous(), w.contiguous(), b, x.new_empty(*x.shape[:-1], w.shape[0]))
        if y is not None:
            return y
    return torch.nn.functional.linear(x, w, b)
