"""Flash attention (varlen, causal/sliding-window, GQA-native) on gfx950 MFMA (``csrc/kernels/flash_*.hip``).

Replaces the reference's CUDA ``flash_attn_varlen_func`` dependency (``attention.py:204-259``).
Layout is token-major ``[T, heads, head_dim]`` with arbitrary token/head strides, so q/k/v can be
strided views of the fused QKV projection (no ``rearrange`` copies, no ``repeat_kv``).
Backward is deterministic (dK/dV and dQ each owned by one workgroup, no float atomics).
"""
from __future__ import annotations

import math
from typing import Any, Optional

import torch

from ._ext import ext, use_native


def attention_reference(q, k, v, cu_q, cu_k, scale, causal, window=-1, dropout_p: float = 0.0, training=False):
    """Dense per-segment fp32 attention (numerical oracle and CPU path). q:[T,Hq,D], k/v:[Tk,Hk,D]."""
    Hq, Hk = q.shape[1], k.shape[1]
    rep = Hq // Hk
    out = torch.empty(q.shape[0], Hq, v.shape[2], dtype=q.dtype, device=q.device)
    cq, ck = cu_q.tolist(), cu_k.tolist()
    for i in range(len(cq) - 1):
        qs, qe, ks, ke = cq[i], cq[i + 1], ck[i], ck[i + 1]
        if qe == qs:
            continue
        qi = q[qs:qe].float().transpose(0, 1)  # [H, Lq, D]
        ki = k[ks:ke].float().repeat_interleave(rep, dim=1).transpose(0, 1)
        vi = v[ks:ke].float().repeat_interleave(rep, dim=1).transpose(0, 1)
        s = torch.matmul(qi, ki.transpose(1, 2)) * scale
        Lq, Lk = qe - qs, ke - ks
        qpos = torch.arange(Lq, device=q.device)[:, None] + (Lk - Lq)
        kpos = torch.arange(Lk, device=q.device)[None, :]
        ok = torch.ones(Lq, Lk, dtype=torch.bool, device=q.device)
        if causal:
            ok &= kpos <= qpos
        if window is not None and window >= 0:
            ok &= kpos >= qpos - window
            if not causal:
                ok &= kpos <= qpos + window
        s = s.masked_fill(~ok, float("-inf"))
        p = torch.softmax(s, dim=-1)
        p = torch.nan_to_num(p, nan=0.0)
        if dropout_p > 0 and training:
            p = torch.nn.functional.dropout(p, dropout_p)
        out[qs:qe] = torch.matmul(p, vi).transpose(0, 1).to(q.dtype)
    return out


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, q, k, v, cu_q, cu_k, max_q, max_k, scale, causal, window):  # type: ignore[override]
        o, lse = ext().fa_fwd(q, k, v, cu_q, cu_k, max_q, scale, causal, window)
        ctx.save_for_backward(q, k, v, o, lse, cu_q, cu_k)
        ctx.cfg = (max_q, max_k, scale, causal, window)
        return o

    @staticmethod
    def backward(ctx: Any, do: torch.Tensor):  # type: ignore[override]
        q, k, v, o, lse, cu_q, cu_k = ctx.saved_tensors
        max_q, max_k, scale, causal, window = ctx.cfg
        dq, dk, dv = ext().fa_bwd(do, q, k, v, o, lse, cu_q, cu_k, max_q, max_k, scale, causal, window)
        return dq, dk, dv, None, None, None, None, None, None, None


def _spec(t: torch.Tensor, base: torch.Tensor) -> tuple:
    return (tuple(t.shape), tuple(t.stride()), t.storage_offset() - base.storage_offset())


def _view(base: torch.Tensor, spec: tuple) -> torch.Tensor:
    shape, stride, off = spec
    return base.as_strided(shape, stride, base.storage_offset() + off)


class _RopeFlashAttn(torch.autograd.Function):
    """RoPE on q/k + flash attention over views of ONE projection output (``base``).

    Backward allocates ``dbase`` once: the attention backward writes dq/dk/dv straight into its q/k/v
    slices and the inverse rotation runs in place there, so no per-slice gradient buffers, zero-fills,
    slice copies or gradient sums are materialised (autograd's view backward would do all of those)."""

    @staticmethod
    def forward(ctx: Any, base, specs, cos, sin, pos, rot_dim, seq_len, interleaved, cu_q, cu_k, max_q, max_k, scale,
                causal, window):  # type: ignore[override]
        qi, ki, vi = (_view(base, sp) for sp in specs)
        q = ext().rope(qi, cos, sin, pos, rot_dim, seq_len, interleaved, False)
        k = ext().rope(ki, cos, sin, pos, rot_dim, seq_len, interleaved, False)
        o, lse = ext().fa_fwd(q, k, vi, cu_q, cu_k, max_q, scale, causal, window)
        ctx.save_for_backward(base, q, k, o, lse, cu_q, cu_k, cos, sin, pos)
        ctx.cfg = (specs, rot_dim, seq_len, interleaved, max_q, max_k, scale, causal, window)
        return o

    @staticmethod
    def backward(ctx: Any, do: torch.Tensor):  # type: ignore[override]
        base, q, k, o, lse, cu_q, cu_k, cos, sin, pos = ctx.saved_tensors
        specs, rot_dim, seq_len, interleaved, max_q, max_k, scale, causal, window = ctx.cfg
        dbase = torch.empty_like(base)
        dq, dk, dv = (_view(dbase, sp) for sp in specs)
        v = _view(base, specs[2])
        ext().fa_bwd(do, q, k, v, o, lse, cu_q, cu_k, max_q, max_k, scale, causal, window, dq, dk, dv)
        ext().rope(dq, cos, sin, pos, rot_dim, seq_len, interleaved, True, dq)
        ext().rope(dk, cos, sin, pos, rot_dim, seq_len, interleaved, True, dk)
        return (dbase,) + (None,) * 14


def rope_flash_attention(base: torch.Tensor, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cos: torch.Tensor,
                         sin: torch.Tensor, pos: Optional[torch.Tensor], rot_dim: int, seq_len: int, interleaved: bool,
                         cu_seqlens: torch.Tensor, max_seqlen: int, softmax_scale: float, causal: bool = True,
                         window: Optional[int] = None) -> Optional[torch.Tensor]:
    """Fused RoPE + flash attention for q/k/v that are views tiling ``base`` exactly (the QKV GEMM output).

    Returns None when the fused path does not apply (CPU tensors, layouts that do not tile ``base``); the
    caller then runs rope and :func:`flash_attention` separately."""
    if not (use_native(base) and base.is_contiguous() and base.dtype == torch.bfloat16):
        return None
    if q.numel() + k.numel() + v.numel() != base.numel():
        return None
    for t in (q, k, v):
        if t.untyped_storage().data_ptr() != base.untyped_storage().data_ptr():
            return None
    specs = (_spec(q, base), _spec(k, base), _spec(v, base))
    cq = cu_seqlens.to(torch.int32)
    p = None if pos is None else pos.reshape(-1).long()
    win = -1 if window is None else int(window)
    return _RopeFlashAttn.apply(base, specs, cos, sin, p, int(rot_dim), int(seq_len), bool(interleaved), cq, cq,
                                int(max_seqlen), int(max_seqlen), float(softmax_scale), bool(causal), win)


def flash_attention(
    q: torch.Tensor,
    k: torch.Tensor,
    v: torch.Tensor,
    cu_seqlens_q: torch.Tensor,
    cu_seqlens_k: Optional[torch.Tensor] = None,
    max_seqlen_q: Optional[int] = None,
    max_seqlen_k: Optional[int] = None,
    softmax_scale: Optional[float] = None,
    causal: bool = True,
    window: Optional[int] = None,
    dropout_p: float = 0.0,
    training: bool = False,
) -> torch.Tensor:
    """q: [T, Hq, D]; k, v: [Tk, Hk, D] (unit last stride); cu_seqlens int32 [nseg+1]."""
    if cu_seqlens_k is None:
        cu_seqlens_k = cu_seqlens_q
        max_seqlen_k = max_seqlen_q
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    win = -1 if window is None else int(window)
    if use_native(q) and dropout_p == 0.0 or (use_native(q) and not training):
        cq = cu_seqlens_q.to(torch.int32)
        ck = cu_seqlens_k.to(torch.int32)
        if max_seqlen_q is None:
            max_seqlen_q = int((cq[1:] - cq[:-1]).max().item())
        if max_seqlen_k is None:
            max_seqlen_k = int((ck[1:] - ck[:-1]).max().item())
        return _FlashAttn.apply(q, k, v, cq, ck, int(max_seqlen_q), int(max_seqlen_k), float(scale), bool(causal), win)
    return attention_reference(q, k, v, cu_seqlens_q, cu_seqlens_k, scale, causal, win, dropout_p, training)
