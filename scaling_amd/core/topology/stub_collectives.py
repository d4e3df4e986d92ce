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

Emulated communication (``SCALING_AMD_PROXY_COMM=emulate``, ``bench.py --proxy-comm emulate``): every stand-in on a GPU
tensor of a group of n > 1 ranks also enqueues what the real collective costs THIS GPU -- ``ext().xgmi_emulate``: the
ring's per-rank send volume streamed through HBM by ``SCALING_AMD_PROXY_COMM_WG`` workgroups (default 16; RCCL's
channels occupy CUs the same way), those CUs then held until the modelled xGMI time
(``comm_estimate.collective_time_s``) has passed.  A blocking collective runs on the caller's current stream (the
framework's communication stream where it chose one); ``async_op=True`` runs it on a proxy stream that waits for the
caller's stream, and ``Work.wait()`` makes the waiting stream wait for it -- RCCL's semantics.  The proxy's step then
contains the communication's interference with the compute (CUs, HBM, stream dependencies), not just its absence.
"""
from __future__ import annotations

import os
from typing import Any

import torch
import torch.distributed as dist

_installed = False
_emu: dict[str, Any] = {}  # emulation settings + per-device scratch ring / proxy stream (empty: stubs only)


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


class _EmuWork:
    """Work handle of an emulated asynchronous collective: ``wait`` makes the current stream wait for it."""

    def __init__(self, ev: Any) -> None:
        self.ev = ev

    def wait(self, timeout: Any = None) -> bool:
        torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self) -> bool:
        return bool(self.ev.query())


def _scratch(dev: torch.device) -> torch.Tensor:
    key = ("scratch", dev.index)
    if key not in _emu:
        _emu[key] = torch.empty(64 << 20, dtype=torch.float32, device=dev)  # 256 MiB ring
    return _emu[key]


def _emulate(kind: str, t: torch.Tensor, full_bytes: int, group: Any, async_op: bool) -> Any:
    """Enqueues the local cost of collective ``kind`` over ``full_bytes`` (see module docstring); returns its handle."""
    n = dist.get_world_size(group)
    if not _emu.get("on") or n <= 1 or not t.is_cuda:
        return _ret(async_op)
    from ...ops._ext import ext
    from ...transformer.utils.comm_estimate import collective_time_s, ring_send_bytes

    us = 1e6 * collective_time_s(kind, full_bytes, n, _emu["eff"])
    send = int(ring_send_bytes(kind, full_bytes, n)) // 16 * 16
    src = t if t.is_contiguous() else t.new_empty(0)
    if not async_op:
        ext().xgmi_emulate(src, _scratch(t.device), send, us, _emu["wg"])
        return None
    cur = torch.cuda.current_stream(t.device)
    key = ("stream", t.device.index)
    side = _emu.setdefault(key, torch.cuda.Stream(device=t.device))
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        ext().xgmi_emulate(src, _scratch(t.device), send, us, _emu["wg"])
        ev = torch.cuda.Event()
        ev.record(side)
    t.record_stream(side)
    return _EmuWork(ev)


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


# Local stand-ins with the tensor semantics of a group whose every rank holds this rank's data (stream-ordered torch
# ops on the current stream; torch's fake backend is not relied on for writing outputs).
def _all_reduce(tensor: torch.Tensor, op: Any = None, group: Any = None, async_op: bool = False) -> Any:
    return _emulate("all_reduce", tensor, _nbytes(tensor), group, async_op)


def _broadcast(tensor: torch.Tensor, src: Any = None, group: Any = None, async_op: bool = False, **_k: Any) -> Any:
    return _emulate("all_gather", tensor, _nbytes(tensor), group, async_op)


def _all_gather_into_tensor(output: torch.Tensor, input: torch.Tensor, group: Any = None, async_op: bool = False) -> Any:
    n = dist.get_world_size(group)
    flat, src = output.view(n, -1), input.reshape(-1)
    for i in range(n):  # contiguous device copies (a broadcast copy_ runs a slow strided elementwise kernel)
        flat[i].copy_(src)
    return _emulate("all_gather", output, _nbytes(output), group, async_op)


def _all_gather(tensor_list: list, tensor: torch.Tensor, group: Any = None, async_op: bool = False) -> Any:
    for t in tensor_list:
        t.copy_(tensor)
    return _emulate("all_gather", tensor, _nbytes(tensor) * len(tensor_list), group, async_op)


def _reduce_scatter_tensor(output: torch.Tensor, input: torch.Tensor, op: Any = None, group: Any = None,
                           async_op: bool = False) -> Any:
    r, n = dist.get_rank(group), output.numel()
    output.view(-1).copy_(input.reshape(-1)[r * n:(r + 1) * n])
    return _emulate("reduce_scatter", input, _nbytes(input), group, async_op)


def _barrier(group: Any = None, async_op: bool = False, **_k: Any) -> Any:
    return _ret(async_op)


def _refuse_p2p(*_a: Any, **_k: Any) -> Any:
    raise RuntimeError("the stubbed (fake) process group has no peers: pipeline parallelism cannot run in the per-rank "
                       "proxy (bench.py --shard-proxy runs one pipeline stage's layers without the pipe)")


def install() -> None:
    """Idempotent: every collective this framework calls gets its local stand-in (plus its emulated cost with
    ``SCALING_AMD_PROXY_COMM=emulate``), p2p is refused."""
    global _installed
    if _installed:
        return
    _installed = True
    mode = os.environ.get("SCALING_AMD_PROXY_COMM", "stub")
    if mode not in ("stub", "emulate"):
        raise ValueError(f"SCALING_AMD_PROXY_COMM={mode!r}: expected 'stub' or 'emulate'")
    _emu.update(on=mode == "emulate", wg=int(os.environ.get("SCALING_AMD_PROXY_COMM_WG", "16")),
                eff=float(os.environ.get("SCALING_AMD_PROXY_COMM_EFF", "0.75")))
    dist.all_reduce = _all_reduce
    dist.broadcast = _broadcast
    dist.all_gather_into_tensor = _all_gather_into_tensor
    dist.all_gather = _all_gather
    dist.reduce_scatter_tensor = _reduce_scatter_tensor
    dist.barrier = _barrier
    dist.batch_isend_irecv = _refuse_p2p
    dist.isend = _refuse_p2p
    dist.irecv = _refuse_p2p
