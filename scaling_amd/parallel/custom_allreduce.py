"""One-shot all-reduce for small tensor-parallel messages over IPC-mapped peer buffers (single node).

Every rank of the process group registers one device buffer (two data slots + a flag row), the IPC handles
are exchanged once over the group, and each rank maps its peers' buffers.  ``__call__(x)`` reduces ``x`` in
place with ONE kernel (``csrc/kernels/oneshot_allreduce.hip``): publish own slot, flag barrier over xGMI,
read-and-sum every rank's slot in a fixed order (bit-identical results on all ranks).  Messages larger than the
slot capacity, or that are not a multiple of 16 bytes, return False and the caller uses RCCL.

Opt-in for tensor parallelism with ``SCALING_AMD_CUSTOM_ALLREDUCE=1`` (``parallel.tp.raw_all_reduce``): the
protocol is exercised by a 2-process test on one GPU; multi-GPU xGMI runs are not covered by the test-suite.

Safety: enabling is a GROUP decision (every rank allocates / maps, then a MIN all-reduce of the per-rank success
flag; all ranks use the path or none does), and a flag-wait timeout in the kernel poisons the output with NaN and
sets the communicator's error word.  Training reads the words once per step on the host (``Optimizer._grad_stats``,
one all-reduce with the grad norm) and raises instead of training on garbage; forward-only use (inference,
``generate``, evaluation steps) calls ``raise_on_errors`` once per call.  After a timeout every communicator is
retired (``disable_all``): its epoch / slot state is out of step across the ranks, so later calls fall back to RCCL.
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
    def __init__(self, group: Any, device: torch.device, capacity_bytes: int = 32 << 20,
                 max_spins: int = 1 << 26) -> None:
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert 1 <= self.world <= 8, "one-shot all-reduce supports up to 8 ranks"
        self.device = device
        self.cap = int(capacity_bytes) // 256 * 256
        dev = device.index if device.index is not None else (torch.cuda.current_device() if device.type == "cuda" else 0)
        self.own: Optional[int] = None
        self.bases: list[int] = []
        self.epoch = 0
        self.max_spins = int(max_spins)  # flag-wait bound per peer (~seconds at the default)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        handle: Optional[bytes] = None
        ok = True
        try:
            self.own, handle = ext().ar_alloc(2 * self.cap + _FLAG_BYTES, dev)
        except Exception:  # noqa: BLE001 - decided collectively below
            ok = False
        infos: list[Any] = [None] * self.world
        dist.all_gather_object(infos, (handle, socket.gethostname()), group=group)  # every rank reaches this
        self.single_node = len({h for _, h in infos}) == 1
        opened: dict[int, int] = {}
        if ok and self.single_node and all(h is not None for h, _ in infos):
            try:
                for i, (h, _) in enumerate(infos):
                    if i != self.rank:
                        opened[i] = ext().ar_open(h, dev)
            except Exception:  # noqa: BLE001
                ok = False
        else:
            ok = False
        if not _group_all(ok, group, device):
            for b in opened.values():
                ext().ar_close(b)
            if self.own is not None:
                if device.type == "cuda":
                    torch.cuda.synchronize(device)
                ext().ar_free(self.own)
            self.own = None
            raise RuntimeError("one-shot all-reduce unavailable on at least one rank of the group")
        self.bases = [self.own if i == self.rank else opened[i] for i in range(self.world)]

    def __call__(self, x: torch.Tensor) -> bool:
        if not (self.single_node and x.is_cuda and x.is_contiguous() and x.nbytes <= self.cap and x.nbytes % 16 == 0
                and x.dtype in (torch.bfloat16, torch.float16, torch.float32)):
            return False
        self.epoch += 1
        slot = (self.epoch & 1) * self.cap
        ext().ar_allreduce(x, self.bases, self.rank, slot, 2 * self.cap, self.epoch, True, self.err, self.max_spins)
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
        if self.own is not None:
            ext().ar_free(self.own)
        self.own = None
        self.bases = []


def _group_all(ok: bool, group: Any, device: torch.device) -> bool:
    """True iff `ok` holds on every rank of `group` (MIN all-reduce; the tensor lives where the backend wants it)."""
    on_gpu = dist.get_backend(group) == "nccl"
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device if on_gpu else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(int(flag.item()) == 1)


def for_group(group: Any, device: torch.device) -> Optional[OneShotAllReduce]:
    """The group's communicator (created on first use, collectively), or None when disabled / not possible.

    Every rank of the group must call this at the same point (it is reached from the same collective call site
    on all ranks); the constructor's success is agreed on collectively, so either all ranks get a communicator or
    all get None and stay on RCCL."""
    if not enabled() or device.type != "cuda":
        return None
    if group not in _REGISTRY:
        try:
            _REGISTRY[group] = OneShotAllReduce(group, device)
        except RuntimeError:  # agreed on by every rank: stay on RCCL everywhere
            _REGISTRY[group] = None
    return _REGISTRY[group]


def pending_error_words() -> list[torch.Tensor]:
    """Device error words of every live communicator (non-zero = a call timed out waiting for a peer)."""
    return [ar.err for ar in _REGISTRY.values() if ar is not None]


def reset_error_words() -> None:
    for ar in _REGISTRY.values():
        if ar is not None:
            ar.err.zero_()


def disable_all() -> None:
    """Retires every communicator after a peer timeout: the group falls back to RCCL from here on (the one-shot
    protocol's epoch / double-buffered slot state is no longer in step across the ranks).  The peer mappings stay
    open until process exit (a rank may still be inside a kernel reading them)."""
    for group in list(_REGISTRY):
        _REGISTRY[group] = None


def _world_max(v: int) -> int:
    """MAX of ``v`` over the whole world (every rank calls this at the same point), ``v`` without a process group."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return v
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def raise_on_errors() -> None:
    """Host check of the error words: raises RuntimeError and retires the communicators if a one-shot all-reduce
    timed out since the last check, on EVERY rank.  For forward-only paths; training checks per step.

    A timeout is often one-sided: the rank that waited sets its word while the late peer saw every flag and finished
    normally.  Deciding on the local word alone would retire the communicator on one rank only, and the two ranks
    would then disagree on the all-reduce path (one on RCCL, one in the one-shot kernel): the next TP all-reduce
    hangs.  So the summed word is MAX all-reduced over the world (as ``Optimizer._grad_stats`` does for training)
    and every rank resets, retires and raises together.  All ranks reach this call at the same point (end of an
    evaluation step / ``run_instructions``); with the path disabled by the environment (same on every rank) it
    costs nothing."""
    if not enabled():
        return
    errs = pending_error_words()
    local = int(torch.stack(errs).sum().item()) if errs else 0
    if _world_max(local) > 0:
        reset_error_words()
        disable_all()
        raise RuntimeError("one-shot tensor-parallel all-reduce timed out waiting for a peer on some rank; its outputs "
                           "were poisoned (NaN); the one-shot path is disabled on every rank, RCCL is used from here on")
