"""Raw tensor / sequence-parallel collectives (no autograd): the RCCL calls behind the region functions of
``core/nn/linear/utils.py`` and the overlapped TP linears (reference ``src/scaling/core/nn/linear/utils.py:254-362``).

Design notes (MI355X): everything bypasses at tp == 1; sequence-parallel shards are contiguous
slices of the *flattened* ``[b*s, h]`` token buffer (as the reference's flat ``reduce_scatter_tensor``
does) so they map to one RCCL reduce-scatter with no repacking; all collectives run on the current
stream — RCCL over a single TP2 xGMI link is latency-bound at these sizes and overlaps best with the
GEMM that produced its input when launched immediately.
"""
from __future__ import annotations

from typing import Any

import torch
import torch.distributed as dist


def tp_of(topology: Any) -> tuple[int, int, Any]:
    """(TP size, TP rank, TP group) of a topology; (1, 0, None) without one or before the process group exists."""
    if topology is None or not getattr(topology, "is_distributed_initialized", False):
        return 1, 0, None
    return topology.config.model_parallel_size, topology.model_parallel_rank, topology.model_parallel_group


def raw_all_reduce(x: torch.Tensor, size: int, group: Any) -> torch.Tensor:
    if size == 1:
        return x
    x = x.contiguous()
    if x.is_cuda:
        from .custom_allreduce import for_group

        ar = for_group(group, x.device)  # opt-in one-shot xGMI all-reduce for small messages
        if ar is not None and ar(x):
            return x
    dist.all_reduce(x, group=group)
    return x


def raw_all_gather_cat(x: torch.Tensor, dim: int, size: int, rank: int, group: Any) -> torch.Tensor:
    if size == 1:
        return x
    x = x.contiguous()
    dim = dim % x.dim()
    if dim == 0:
        out = torch.empty((x.shape[0] * size,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out
    # gather into a leading "rank" axis (one contiguous collective), then move it next to `dim`
    buf = torch.empty((size,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(buf.view(-1), x.view(-1), group=group)
    parts = list(buf.unbind(0))
    return torch.cat(parts, dim=dim)


def raw_shard(x: torch.Tensor, dim: int, size: int, rank: int) -> torch.Tensor:
    if size == 1:
        return x
    n = x.shape[dim] // size
    return x.narrow(dim, rank * n, n).contiguous()


def raw_reduce_scatter_seq(x: torch.Tensor, size: int, group: Any) -> torch.Tensor:
    """Sum over the TP group and keep this rank's 1/size of the tokens; [b, s, ...] -> [b, s/size, ...].

    Operates on the flattened buffer (rank r keeps the r-th contiguous chunk), which is the partition
    RCCL's reduce-scatter produces; the sequence-parallel region is token-wise so only the consistency
    of scatter and gather matters (reference ``core/nn/linear/utils.py:270-310``)."""
    if size == 1:
        return x
    shape = list(x.shape)
    assert shape[1] % size == 0, "Sequence parallel size should be divisible by tensor parallel size"
    shape[1] //= size
    out = torch.empty(shape, dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out.view(-1), x.contiguous().view(-1), group=group)
    return out


def raw_gather_seq(x: torch.Tensor, size: int, group: Any) -> torch.Tensor:
    if size == 1:
        return x
    shape = list(x.shape)
    shape[1] *= size
    out = torch.empty(shape, dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out.view(-1), x.contiguous().view(-1), group=group)
    return out
