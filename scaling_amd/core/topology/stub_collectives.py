"""Stubbed collectives for the 1-GPU per-rank proxy (``TopologyConfig.backend = "fake"``, ``bench.py --shard-proxy``).

One process plays rank 0 of a tensor-parallel world: every layer is built with its per-rank shard shapes (TP2: 16 of 32
query heads, 4 of 8 KV heads, SwiGLU 5504 of 11008, vocab 16000 of 32000) and runs exactly the kernels one rank of the
real layout runs, while the collectives between the ranks are replaced by local stand-ins of the same tensor shapes
(torch's ``fake`` process-group backend; no peer exists).  So the per-rank COMPUTE of a layout (GEMM shapes, attention
head split, HIP vs vendor kernel routing, activation checkpointing cost) is measurable on one GPU; communication time
is not in it.

``fake``'s own semantics: all-reduce and broadcast leave the tensor unchanged, all-gather writes the local input into
every rank's slot.  Its reduce-scatter leaves the output unwritten (uninitialised memory): ``install`` makes it copy
this rank's slice of the input instead.  Point-to-point messages have no peer, so pipeline parallelism is refused.
"""
from __future__ import annotations

import functools
from typing import Any, Callable

import torch
import torch.distributed as dist

_installed = False


def init_fake_process_group(world_size: int, rank: int) -> None:
    from torch.testing._internal.distributed.fake_pg import FakeStore

    dist.init_process_group("fake", store=FakeStore(), world_size=world_size, rank=rank)


def _wrap_reduce_scatter(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(output: torch.Tensor, input: torch.Tensor, op: Any = None, group: Any = None, async_op: bool = False) -> Any:
        r, n = dist.get_rank(group), output.numel()
        output.view(-1).copy_(input.reshape(-1)[r * n:(r + 1) * n])
        return None

    return fn


def _refuse_p2p(*_a: Any, **_k: Any) -> Any:
    raise RuntimeError("the stubbed (fake) process group has no peers: pipeline parallelism cannot run in the per-rank "
                       "proxy (bench.py --shard-proxy runs one pipeline stage's layers without the pipe)")


def install() -> None:
    """Idempotent: local reduce-scatter semantics, p2p refused."""
    global _installed
    if _installed:
        return
    _installed = True
    dist.reduce_scatter_tensor = _wrap_reduce_scatter(dist.reduce_scatter_tensor)
    dist.batch_isend_irecv = _refuse_p2p
    dist.isend = _refuse_p2p
    dist.irecv = _refuse_p2p
