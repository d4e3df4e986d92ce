"""Fused (vocab-parallel) cross-entropy on bf16 logits (``csrc/kernels/xent_embed_optim.hip``).

One pass computes per-row (max, sum-exp, target logit, argmax) without materialising fp32 logits
(the reference upcasts ``[b*s, V]`` to fp32, ``transformer/model/model.py:56-76``).  With tensor
parallelism each rank holds ``[N, V/tp]`` and the row statistics are combined with three small
all-reduces — the full-vocab logits are never all-gathered.  The backward writes
``(softmax - onehot) * dloss`` in place over the logits buffer.
"""
from __future__ import annotations

from typing import Any, Optional

import torch
import torch.distributed as dist

from ._ext import ext, use_native


def _combine(m, s, t, am, group, tp):
    if tp == 1:
        return m + torch.log(s), t, am
    gm = m.clone()
    dist.all_reduce(gm, op=dist.ReduceOp.MAX, group=group)
    s = s * torch.exp(m - gm)
    dist.all_reduce(s, group=group)
    dist.all_reduce(t, group=group)
    # argmax across shards: smallest global index among shards attaining the max
    cand = torch.where(m == gm, am, torch.full_like(am, torch.iinfo(torch.int64).max))
    dist.all_reduce(cand, op=dist.ReduceOp.MIN, group=group)
    return gm + torch.log(s), t, cand


class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, logits: torch.Tensor, target: torch.Tensor, v0: int, group: Any, tp: int,
                inplace_grad: bool):  # type: ignore[override]
        lg = logits.reshape(-1, logits.shape[-1])
        if not lg.is_contiguous():
            lg = lg.contiguous()
        tgt = target.reshape(-1)
        m, s, t, am = ext().xent_stats(lg, tgt, v0)
        lse, tl, amax = _combine(m, s, t, am, group, tp)
        loss = lse - tl
        ctx.save_for_backward(lg, tgt, lse)
        ctx.v0, ctx.inplace, ctx.shape = v0, inplace_grad, logits.shape
        ctx.mark_non_differentiable(amax)
        return loss.view(target.shape), amax.view(target.shape)

    @staticmethod
    def backward(ctx: Any, gloss: torch.Tensor, _g2: Optional[torch.Tensor]):  # type: ignore[override]
        lg, tgt, lse = ctx.saved_tensors
        g = gloss.reshape(-1).float().contiguous()
        d = ext().xent_bwd(lg, tgt, lse, g, ctx.v0, ctx.inplace)
        return d.view(ctx.shape), None, None, None, None, None


def cross_entropy_reference(logits: torch.Tensor, target: torch.Tensor, v0: int = 0, group: Any = None, tp: int = 1):
    lf = logits.float()
    if tp == 1:
        loss = torch.nn.functional.cross_entropy(lf.reshape(-1, lf.shape[-1]), target.reshape(-1), reduction="none")
        return loss.view(target.shape), lf.argmax(-1)
    # vocab-parallel reference in plain torch
    V = lf.shape[-1]
    m = lf.max(-1).values
    gm = m.detach().clone()
    dist.all_reduce(gm, op=dist.ReduceOp.MAX, group=group)
    e = torch.exp(lf - gm.unsqueeze(-1))
    s = e.sum(-1)
    s = _AllReduceSum.apply(s, group)
    local = target - v0
    inr = (local >= 0) & (local < V)
    tl = torch.gather(lf, -1, local.clamp(0, V - 1).unsqueeze(-1)).squeeze(-1) * inr
    tl = _AllReduceSum.apply(tl, group)
    loss = gm + torch.log(s) - tl
    mv, mi = lf.max(-1)
    gmv = mv.detach().clone()
    dist.all_reduce(gmv, op=dist.ReduceOp.MAX, group=group)
    cand = torch.where(mv == gmv, mi + v0, torch.full_like(mi, torch.iinfo(torch.int64).max))
    dist.all_reduce(cand, op=dist.ReduceOp.MIN, group=group)
    return loss, cand


class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, group: Any) -> torch.Tensor:  # type: ignore[override]
        y = x.clone()
        dist.all_reduce(y, group=group)
        return y

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        return g, None


def vocab_parallel_cross_entropy(logits: torch.Tensor, target: torch.Tensor, v0: int = 0, group: Any = None,
                                 tp: int = 1, inplace_grad: bool = False):
    """Returns (per-token loss fp32, argmax token id).  ``logits`` holds vocab rows [v0, v0 + V_local)."""
    if use_native(logits):
        return _XEnt.apply(logits, target, v0, group, tp, inplace_grad)
    return cross_entropy_reference(logits, target, v0, group, tp)
