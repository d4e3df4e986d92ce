"""Stubbed collectives for the 1-GPU per-rank proxy (``TopologyConfig.backend = "fake"``, ``bench.py --shard-proxy``).

One process plays rank 0 of a tensor-parallel world: every layer is built with its per-rank shard shapes (TP2: 16 of 32
query heads, 4 of 8 KV heads, SwiGLU 5504 of 11008, vocab 16000 of 32000) and runs exactly the kernels one rank of the
real layout runs, while the collectives between the ranks are replaced by local stand-ins of the same tensor shapes
(torch's ``fake`` process-group backend; no peer exists).  So the per-rank COMPUTE of a layout (GEMM shapes, attention
head split, HIP vs vendor kernel routing, activation checkpointing cost) is measurable on one GPU; communication time
is not in it.

``install`` replaces every collective this framework calls by a local stand-in with the semantics of a group whose
ranks all hold this rank's data: all-reduce / broadcast / barrier do nothing, all-gather replicates the local input
into every slot, reduce-scatter copies this rank's slice of the input (torch's ``fake`` backend only provides the
process-group plumbing; on GPU tensors it leaves outputs unwritten, which made the first proxy run diverge to NaN).
Point-to-point messages have no peer, so pipeline parallelism is refused.
"""
from __future__ import annotations

from typing import Any

import torch
import torch.distributed as dist

_installed = False


def init_fake_process_group(world_size: int, rank: int) -> None:
    from torch.testing._internal.distributed.fake_pg import FakeStore

    dist.init_process_group("fake", store=FakeStore(), world_size=world_size, rank=rank)


class _Done:
    def wait(self, timeout: Any = None) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


def _ret(async_op: bool) -> Any:
    return _Done() if async_op else None


# Local stand-ins with the tensor semantics of a group whose every rank holds this rank's data (stream-ordered torch
# ops on the current stream; torch's fake backend is not relied on for writing outputs).
def _all_reduce(tensor: torch.Tensor, op: Any = None, group: Any = None, async_op: bool = False) -> Any:
    return _ret(async_op)


def _broadcast(tensor: torch.Tensor, src: Any = None, group: Any = None, async_op: bool = False, **_k: Any) -> Any:
    return _ret(async_op)


def _all_gather_into_tensor(output: torch.Tensor, input: torch.Tensor, group: Any = None, async_op: bool = False) -> Any:
    n = dist.get_world_size(group)
    flat, src = output.view(n, -1), input.reshape(-1)
    for i in range(n):  # contiguous device copies (a broadcast copy_ runs a slow strided elementwise kernel)
        flat[i].copy_(src)
    return _ret(async_op)


def _all_gather(tensor_list: list, tensor: torch.Tensor, group: Any = None, async_op: bool = False) -> Any:
    for t in tensor_list:
        t.copy_(tensor)
    return _ret(async_op)


def _reduce_scatter_tensor(output: torch.Tensor, input: torch.Tensor, op: Any = None, group: Any = None,
                           async_op: bool = False) -> Any:
    r, n = dist.get_rank(group), output.numel()
    output.view(-1).copy_(input.reshape(-1)[r * n:(r + 1) * n])
    return _ret(async_op)


def _barrier(group: Any = None, async_op: bool = False, **_k: Any) -> Any:
    return _ret(async_op)


def _refuse_p2p(*_a: Any, **_k: Any) -> Any:
    raise RuntimeError("the stubbed (fake) process group has no peers: pipeline parallelism cannot run in the per-rank "
                       "proxy (bench.py --shard-proxy runs one pipeline stage's layers without the pipe)")


def install() -> None:
    """Idempotent: every collective this framework calls gets its local stand-in, p2p is refused."""
    global _installed
    if _installed:
        return
    _installed = True
    dist.all_reduce = _all_reduce
    dist.broadcast = _broadcast
    dist.all_gather_into_tensor = _all_gather_into_tensor
    dist.all_gather = _all_gather
    dist.reduce_scatter_tensor = _reduce_scatter_tensor
    dist.barrier = _barrier
    dist.batch_isend_irecv = _refuse_p2p
    dist.isend = _refuse_p2p
    dist.irecv = _refuse_p2p
