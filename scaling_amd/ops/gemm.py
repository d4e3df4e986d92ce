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

``linear`` is the forward ``x W^T (+ b)`` of every linear layer and ``mm_nt`` the input gradient ``dY (W^T)^T`` on
the cached transpose: at most 4 token rows (token-by-token decoding) run the weight-streaming GEMV kernel
(``csrc/kernels/gemv.hip``); larger products run the HIP NT kernel (``csrc/kernels/gemm_nt.hip``) where
``nt_enabled`` says so, else hipBLASLt.  ``SCALING_AMD_NT_GEMM``: ``1`` = the HIP kernel for every shape it tiles,
``0`` = hipBLASLt everywhere, ``auto`` (default) = the HIP kernel for the (N, K) shapes in ``NT_FASTER`` (measured
faster than hipBLASLt's tuned solution on MI355X, ``tools/gemm_nt_bench.py``).
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

_NT_MODE = os.environ.get("SCALING_AMD_NT_GEMM", "auto")
# (N out, K in) shapes of y = x W^T where the HIP NT kernel beat hipBLASLt (tools/gemm_nt_bench.py, MI355X)
NT_FASTER: set[tuple[int, int]] = set()


# (2F, H) gate/up weight shapes where the one-node SwiGLU MLP on the NT kernel's fused epilogues (forward z / h,
# backward dz) beat hipBLASLt + the stand-alone SwiGLU kernels, forward + backward together (tools/gemm_nt_bench.py).
# Empty: at the 7B shape (22016, 4096) the fused backward is 1.2-1.4 % faster but the fused forward 1.5 % slower,
# net +0.03 ms per layer (profiles/gemm_nt_swiglu_bwd_pipelined_r4.log)
NT_FUSED_MLP: set[tuple[int, int]] = set()


def nt_fused_mlp_enabled(a: torch.Tensor, wgu: torch.Tensor) -> bool:
    """Whether the SwiGLU MLP on ``a`` with gate/up weights ``wgu`` ([2F, H]) runs as the fused NT-kernel node
    (policy as ``nt_enabled``, own shape table ``NT_FUSED_MLP``; the node's plain GEMMs still follow ``nt_enabled``)."""
    if _NT_MODE == "0" or not (a.is_cuda and a.dim() == 2 and a.dtype == wgu.dtype == torch.bfloat16):
        return False
    if _NT_MODE != "1" and (int(wgu.shape[0]), int(wgu.shape[1])) not in NT_FUSED_MLP:
        return False
    return bool(ext().gemm_nt_ok(a, wgu))


# (F, H) down-projection shapes where the backward's dh = dY W_down GEMM with the SwiGLU backward in its epilogue
# (``gemm_nt_swiglu_bwd``: writes dz, no dh round trip, no stand-alone SwiGLU backward pass; used with the unfused
# forward) beats hipBLASLt + the SwiGLU backward kernel.  Empty: isolated, the 7B shape (11008, 4096) measured 2.576 vs
# 2.606 ms per layer (profiles/gemm_nt_swiglu_bwd_pipelined_r4.log), but inside the training step the NT kernel takes
# 84.7 ms per step against ~72 ms for what it replaces and the step is 1-2 ms slower (interleaved A/B,
# profiles/swiglu_bwd_nt_ab_r5.log).  SCALING_AMD_SWIGLU_BWD_NT=1 turns it on for every shape the kernel tiles.
NT_SWIGLU_BWD: set[tuple[int, int]] = set()
_SWIGLU_BWD_MODE = os.environ.get("SCALING_AMD_SWIGLU_BWD_NT", "auto")


def nt_swiglu_bwd_enabled(dy_like: torch.Tensor, wdt_shape: tuple[int, int]) -> bool:
    """Policy: whether the SwiGLU backward rides on the NT kernel's dz epilogue for dY shaped like ``dy_like`` ([T, H])
    and ``W_down^T`` of shape ``wdt_shape`` ([F, H]); ``SCALING_AMD_SWIGLU_BWD_NT``: 1 = every shape (the caller still
    checks that the kernel tiles it, ``gemm_nt_ok``), 0 = never, auto = the shapes in ``NT_SWIGLU_BWD``."""
    if _SWIGLU_BWD_MODE == "0" or not (dy_like.is_cuda and dy_like.dim() == 2 and dy_like.dtype == torch.bfloat16):
        return False
    return _SWIGLU_BWD_MODE == "1" or tuple(wdt_shape) in NT_SWIGLU_BWD


def nt_enabled(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Whether ``a @ b^T`` (2-D, b = [N, K]) runs on the HIP NT kernel (policy above + the kernel's tiling)."""
    if _NT_MODE == "0" or not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2):
        return False
    if _NT_MODE != "1" and (int(b.shape[0]), int(b.shape[1])) not in NT_FASTER:
        return False
    return bool(ext().gemm_nt_ok(a, b))


def mm_nt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b^T`` for 2-D ``a`` [M, K] and ``b`` [N, K] (no autograd graph): HIP NT kernel or hipBLASLt."""
    if nt_enabled(a, b):
        out = torch.empty(a.shape[0], b.shape[0], device=a.device, dtype=a.dtype)
        ext().gemm_nt(a, b, out)
        return out
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
    if b is None and not needs_graph and rows > GEMV_MAX_ROWS and w.dim() == 2 and use_native(x):
        x2 = x.reshape(rows, K)
        if nt_enabled(x2, w):
            return mm_nt(x2, w).reshape(*x.shape[:-1], w.shape[0])
    return torch.nn.functional.linear(x, w, b)
