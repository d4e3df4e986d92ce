"""Tensor / sequence-parallel regions as autograd functions (reference ``src/scaling/core/nn/linear/utils.py:20-251``).

Megatron region semantics:

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

Each region is one generic autograd node whose forward and backward are raw collectives of ``parallel/tp.py`` (one
RCCL call each, on the current stream); everything is the identity at TP 1.
"""
from __future__ import annotations

from typing import Any, Callable

import torch

from ....parallel.tp import (  # noqa: F401  (raw collectives re-exported under the reference's module)
    raw_all_gather_cat,
    raw_all_reduce,
    raw_gather_seq,
    raw_reduce_scatter_seq,
    raw_shard,
    tp_of,
)


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
    size, _, group = tp_of(topology)
    if size == 1:
        return x
    return _Region.apply(x, _identity, lambda g: raw_all_reduce(g, size, group))


def all_reduce(x: torch.Tensor, topology: Any) -> torch.Tensor:
    size, _, group = tp_of(topology)
    if size == 1:
        return x
    return _Region.apply(x, lambda t: raw_all_reduce(t.clone(), size, group), _identity)


def all_concat(x: torch.Tensor, dim: int, topology: Any) -> torch.Tensor:
    size, rank, group = tp_of(topology)
    if size == 1:
        return x
    return _Region.apply(
        x, lambda t: raw_all_gather_cat(t, dim, size, rank, group), lambda g: raw_shard(g, dim, size, rank)
    )


def all_shard(x: torch.Tensor, dim: int, topology: Any) -> torch.Tensor:
    size, rank, group = tp_of(topology)
    if size == 1:
        return x
    return _Region.apply(
        x, lambda t: raw_shard(t, dim, size, rank), lambda g: raw_all_gather_cat(g, dim, size, rank, group)
    )


def all_reduce_scatter_to_sequence_parallel(x: torch.Tensor, topology: Any) -> torch.Tensor:
    size, _, group = tp_of(topology)
    if size == 1:
        return x
    return _Region.apply(x, lambda t: raw_reduce_scatter_seq(t, size, group), lambda g: raw_gather_seq(g, size, group))


def gather_from_sequence_parallel_region(
    x: torch.Tensor, topology: Any, tensor_parallel_output_grad: bool = True
) -> torch.Tensor:
    size, _, group = tp_of(topology)
    if size == 1:
        return x
    # both branches reduce-scatter in the reference (utils.py:177-192)
    return _Region.apply(x, lambda t: raw_gather_seq(t, size, group), lambda g: raw_reduce_scatter_seq(g, size, group))


def tp_input_grad_group(topology: Any) -> Any:
    """The TP group whose sum a column-parallel linear's input gradient needs (the ``copy_to`` region's
    backward), or None: tp == 1, sequence parallelism (the gather region in front of the linear reduces
    instead), or no process group."""
    size, _, group = tp_of(topology)
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
