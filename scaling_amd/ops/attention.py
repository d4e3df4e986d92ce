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
