"""One-shot all-reduce for small tensor-parallel messages over IPC-mapped peer buffers (single node).

Every rank of the process group registers one device buffer (two data slots + a flag row), the IPC handles
are exchanged once over the group, and each rank maps its peers' buffers.  ``__call__(x)`` reduces ``x`` in
place with ONE kernel (``csrc/kernels/oneshot_allreduce.hip``): publish own slot, flag barrier over xGMI,
read-and-sum every rank's slot in a fixed order (bit-identical results on all ranks).  Messages larger than the
slot capacity, or that are not a multiple of 16 bytes, return False and the caller uses RCCL.

Opt-in for tensor parallelism with ``SCALING_AMD_CUSTOM_ALLREDUCE=1`` (``parallel.tp.raw_all_reduce``): the
protocol is exercised by a 2-process test on one GPU; multi-GPU xGMI runs are not covered by the test-suite.
"""
from __future__ import annotations

import os
import socket
from typing import Any, Optional

import torch
import torch.distributed as dist

from ..ops._ext import ext

_FLAG_BYTES = 256
_REGISTRY: dict[Any, Optional["OneShotAllReduce"]] = {}


def enabled() -> bool:
    return os.environ.get("SCALING_AMD_CUSTOM_ALLREDUCE", "0") == "1"


class OneShotAllReduce:
    def __init__(self, group: Any, device: torch.device, capacity_bytes: int = 32 << 20) -> None:
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert 1 <= self.world <= 8, "one-shot all-reduce supports up to 8 ranks"
        self.device = device
        self.cap = int(capacity_bytes) // 256 * 256
        dev = device.index if device.index is not None else torch.cuda.current_device()
        self.own, handle = ext().ar_alloc(2 * self.cap + _FLAG_BYTES, dev)
        info = (handle, socket.gethostname())
        infos: list[Any] = [None] * self.world
        dist.all_gather_object(infos, info, group=group)
        self.single_node = len({h for _, h in infos}) == 1
        self.bases = [self.own if i == self.rank else ext().ar_open(h, dev) for i, (h, _) in enumerate(infos)]
        self.epoch = 0
        self.err = torch.zeros(1, dtype=torch.int32, device=device)

    def __call__(self, x: torch.Tensor) -> bool:
        if not (self.single_node and x.is_cuda and x.is_contiguous() and x.nbytes <= self.cap and x.nbytes % 16 == 0
                and x.dtype in (torch.bfloat16, torch.float16, torch.float32)):
            return False
        self.epoch += 1
        slot = (self.epoch & 1) * self.cap
        ext().ar_allreduce(x, self.bases, self.rank, slot, 2 * self.cap, self.epoch, True, self.err)
        return True

    def check(self) -> None:
        """Raises if any call timed out waiting for a peer (host sync: call outside hot loops)."""
        if int(self.err.item()) != 0:
            raise RuntimeError("one-shot all-reduce: a peer did not arrive (timeout)")

    def close(self) -> None:
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        for i, b in enumerate(self.bases):
            if i != self.rank:
                ext().ar_close(b)
        dist.barrier(group=self.group)
        ext().ar_free(self.own)
        self.bases = []


def for_group(group: Any, device: torch.device) -> Optional[OneShotAllReduce]:
    """The group's communicator (created on first use, collectively), or None when disabled / not possible."""
    if not enabled() or device.type != "cuda":
        return None
    if group not in _REGISTRY:
        try:
            _REGISTRY[group] = OneShotAllReduce(group, device)
        except Exception:  # noqa: BLE001 - IPC unavailable: stay on RCCL
            _REGISTRY[group] = None
    return _REGISTRY[group]
