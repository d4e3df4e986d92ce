"""Tensor/sequence-parallel region collectives as autograd functions.

Megatron region semantics (same forward/backward pairs as reference
``src/scaling/core/nn/linear/utils.py:20-251``):

=============================  ==========================  ==========================
region                         forward                     backward
=============================  ==========================  ==========================
copy_to                        identity                    all-reduce
all_concat(dim)                all-gather + cat            take own shard
all_reduce                     all-reduce                  identity
all_shard(dim)                 take own shard              all-gather + cat
reduce_scatter_to_sp           reduce-scatter (dim 1)      all-gather (dim 1)
gather_from_sp                 all-gather (dim 1)          reduce-scatter (dim 1)
=============================  ==========================  ==========================

Design notes (MI355X): everything bypasses at tp == 1; sequence-parallel shards are contiguous
slices of the *flattened* ``[b*s, h]`` token buffer (as the reference's flat ``reduce_scatter_tensor``
does) so they map to one RCCL reduce-scatter with no repacking; all collectives run on the current
stream — RCCL over a single TP2 xGMI link is latency-bound at these sizes and overlaps best with the
GEMM that produced its input when launched immediately.
"""
from __future__ import annotations

from typing import Any, Callable

import torch
import torch.distributed as dist


def _tp(topology: Any) -> tuple[int, int, Any]:
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


class _Region(torch.autograd.Function):
    """Generic region: forward op / backward op chosen by the caller (keeps one autograd class)."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, fwd: Callable, bwd: Callable) -> torch.Tensor:  # type: ignore[override]
        ctx.bwd = bwd
        return fwd(x)

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor) -> tuple:  # type: ignore[override]
        return ctx.bwd(g), None, None


def _identity(x: torch.Tensor) -> torch.Tensor:
    return x


def copy_to_tensor_model_parallel_region(x: torch.Tensor, topology: Any) -> torch.Tensor:
    size, _, group = _tp(topology)
    if size == 1:
        return x
    return _Region.apply(x, _identity, lambda g: raw_all_reduce(g, size, group))


def all_reduce(x: torch.Tensor, topology: Any) -> torch.Tensor:
    size, _, group = _tp(topology)
    if size == 1:
        return x
    return _Region.apply(x, lambda t: raw_all_reduce(t.clone(), size, group), _identity)


def all_concat(x: torch.Tensor, dim: int, topology: Any) -> torch.Tensor:
    size, rank, group = _tp(topology)
    if size == 1:
        return x
    return _Region.apply(
        x, lambda t: raw_all_gather_cat(t, dim, size, rank, group), lambda g: raw_shard(g, dim, size, rank)
    )


def all_shard(x: torch.Tensor, dim: int, topology: Any) -> torch.Tensor:
    size, rank, group = _tp(topology)
    if size == 1:
        return x
    return _Region.apply(
        x, lambda t: raw_shard(t, dim, size, rank), lambda g: raw_all_gather_cat(g, dim, size, rank, group)
    )


def all_reduce_scatter_to_sequence_parallel(x: torch.Tensor, topology: Any) -> torch.Tensor:
    size, _, group = _tp(topology)
    if size == 1:
        return x
    return _Region.apply(x, lambda t: raw_reduce_scatter_seq(t, size, group), lambda g: raw_gather_seq(g, size, group))


def gather_from_sequence_parallel_region(
    x: torch.Tensor, topology: Any, tensor_parallel_output_grad: bool = True
) -> torch.Tensor:
    size, _, group = _tp(topology)
    if size == 1:
        return x
    # both branches reduce-scatter in the reference (utils.py:177-192)
    return _Region.apply(x, lambda t: raw_gather_seq(t, size, group), lambda g: raw_reduce_scatter_seq(g, size, group))


def tp_input_grad_group(topology: Any) -> Any:
    """The TP group whose sum a column-parallel linear's input gradient needs (the ``copy_to`` region's
    backward), or None: tp == 1, sequence parallelism (the gather region in front of the linear reduces
    instead), or no process group."""
    size, _, group = _tp(topology)
    if size == 1 or topology.config.sequence_parallel:
        return None
    return group


def get_device(topology: Any = None, device: torch.device | None = None) -> torch.device:
    assert topology is None or device is None, "cannot specify both device and topology"
    if topology is not None:
        return topology.device
    if device is not None:
        return torch.device(device)
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
