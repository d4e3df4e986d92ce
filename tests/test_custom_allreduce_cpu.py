"""One-shot all-reduce enablement is a group decision (CPU / gloo): if mapping a peer buffer fails on one rank,
EVERY rank falls back to RCCL (no rank spins on IPC flags while another uses the collective), and the buffers
that were allocated / opened are released on every rank."""
from __future__ import annotations

import os

import torch

from tests.dist_utils import run_distributed


class _FakeExt:
    def __init__(self, fail_open_on: int, rank: int) -> None:
        self.fail_open_on, self.rank = fail_open_on, rank
        self.freed: list[int] = []
        self.closed: list[int] = []

    def ar_alloc(self, nbytes: int, dev: int):
        return 1000 + self.rank, b"h%d" % self.rank

    def ar_open(self, handle: bytes, dev: int) -> int:
        if self.rank == self.fail_open_on:
            raise RuntimeError("hipIpcOpenMemHandle failed")
        return 2000 + int(handle[1:])

    def ar_close(self, ptr: int) -> None:
        self.closed.append(ptr)

    def ar_free(self, ptr: int) -> None:
        self.freed.append(ptr)


def _worker(fail_open_on: int):
    import torch.distributed as dist

    from scaling_amd.parallel import custom_allreduce as ca

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    fake = _FakeExt(fail_open_on, rank)
    ca.ext = lambda: fake  # type: ignore[assignment]
    try:
        comm = ca.OneShotAllReduce(dist.group.WORLD, torch.device("cpu"), capacity_bytes=1 << 16)
        got = "enabled"
        assert comm.bases
    except RuntimeError:
        got = "fallback"
    dist.destroy_process_group()
    return got, fake.freed, fake.closed


def test_enablement_is_collective_when_one_rank_fails():
    res = run_distributed(_worker, 3, timeout=120, fail_open_on=1)
    assert {r[0] for r in res.values()} == {"fallback"}
    for rank, (_, freed, closed) in res.items():
        assert freed == [1000 + rank]  # own buffer released everywhere
    # ranks that mapped peers unmapped them again
    assert sorted(res[0][2]) == [2001, 2002] and res[1][2] == [] and sorted(res[2][2]) == [2000, 2001]


def test_enablement_succeeds_when_all_ranks_succeed():
    res = run_distributed(_worker, 2, timeout=120, fail_open_on=-1)
    assert {r[0] for r in res.values()} == {"enabled"}
    assert all(not r[1] and not r[2] for r in res.values())


def test_error_word_raises_and_retires_communicators(monkeypatch):
    """A set error word (a peer timeout) makes ``raise_on_errors`` (forward-only paths) raise, clears the word and
    retires every communicator, so later calls use RCCL instead of the out-of-step one-shot protocol."""
    import pytest

    from scaling_amd.parallel import custom_allreduce as ca

    monkeypatch.setenv("SCALING_AMD_CUSTOM_ALLREDUCE", "1")

    class _Comm:
        def __init__(self) -> None:
            self.err = torch.zeros(1, dtype=torch.int32)

    saved = dict(ca._REGISTRY)
    try:
        ca._REGISTRY.clear()
        a, b = _Comm(), _Comm()
        ca._REGISTRY.update({"g0": a, "g1": b})
        ca.raise_on_errors()  # healthy: no-op
        assert ca._REGISTRY["g0"] is a
        b.err.fill_(1)
        with pytest.raises(RuntimeError, match="timed out"):
            ca.raise_on_errors()
        assert int(b.err.item()) == 0
        assert ca._REGISTRY == {"g0": None, "g1": None}
        assert ca.pending_error_words() == []
    finally:
        ca._REGISTRY.clear()
        ca._REGISTRY.update(saved)


def _one_sided_worker(bad_rank: int):
    import torch.distributed as dist

    from scaling_amd.parallel import custom_allreduce as ca

    os.environ["SCALING_AMD_CUSTOM_ALLREDUCE"] = "1"
    dist.init_process_group("gloo")
    rank = dist.get_rank()

    class _Comm:
        def __init__(self) -> None:
            self.err = torch.zeros(1, dtype=torch.int32)

    c = _Comm()
    ca._REGISTRY.clear()
    ca._REGISTRY["tp"] = c
    ca.raise_on_errors()  # healthy everywhere: no rank raises
    healthy = ca._REGISTRY["tp"] is c
    if rank == bad_rank:  # only the rank that waited saw the timeout; its late peer finished normally
        c.err.fill_(1)
    raised = False
    try:
        ca.raise_on_errors()
    except RuntimeError:
        raised = True
    retired = ca._REGISTRY["tp"] is None
    dist.destroy_process_group()
    return healthy, raised, retired, int(c.err.item())


def test_one_sided_timeout_retires_communicators_on_every_rank():
    """A timeout seen by one rank only must still make EVERY rank raise and fall back to RCCL: deciding on the local
    word would leave the ranks on different all-reduce paths and hang the next TP all-reduce."""
    res = run_distributed(_one_sided_worker, 2, timeout=120, bad_rank=1)
    assert all(r == (True, True, True, 0) for r in res.values()), res
