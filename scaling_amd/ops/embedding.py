"""Vocab-parallel embedding lookup: masked gather forward, deterministic sorted segment-sum backward."""
from __future__ import annotations

from typing import Any

import torch

from ._ext import ext, use_native


class _Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, ids: torch.Tensor, W: torch.Tensor, v0: int) -> torch.Tensor:  # type: ignore[override]
        ctx.save_for_backward(ids)
        ctx.v0 = v0
        ctx.rows = W.shape[0]
        return ext().embed_fwd(ids, W, v0)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor) -> tuple:  # type: ignore[override]
        (ids,) = ctx.saved_tensors
        dW = ext().embed_bwd(dy.reshape(-1, dy.shape[-1]), ids, ctx.rows, ctx.v0)
        return None, dW, None


def vocab_embedding_reference(ids: torch.Tensor, W: torch.Tensor, v0: int, v1: int) -> torch.Tensor:
    if v0 == 0 and v1 == W.shape[0] + v0 and bool(((ids >= v0) & (ids < v1)).all()):
        return torch.nn.functional.embedding(ids, W)
    mask = (ids < v0) | (ids >= v1)
    local = (ids - v0).masked_fill(mask, 0)
    out = torch.nn.functional.embedding(local, W)
    return out.masked_fill(mask.unsqueeze(-1), 0.0)


def vocab_embedding(ids: torch.Tensor, W: torch.Tensor, v0: int, v1: int) -> torch.Tensor:
    if use_native(W) and W.shape[1] % 8 == 0:
        return _Embed.apply(ids, W, v0)
    return vocab_embedding_reference(ids, W, v0, v1)
