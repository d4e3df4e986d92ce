"""One-shot all-reduce over IPC-mapped buffers (GPU): reduction math with several registered buffers in one
process, and the full protocol (IPC handle exchange, flag barrier, double-buffered slots) between two
processes sharing one MI355X."""
from __future__ import annotations

import pytest
import torch

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.gpu


def _ext():
    from scaling_amd.ops._ext import ext

    return ext()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_oneshot_reduction_math_single_process(world, dtype):
    """`world` registered buffers on one device stand in for the peers; no barrier (signal=False)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    cap = 1 << 20
    e = _ext()
    bufs = [e.ar_alloc(2 * cap + 256, 0)[0] for _ in range(world)]
    try:
        torch.manual_seed(0)
        xs = [torch.randn(4096 + 8 * 37, device="cuda", dtype=dtype) for _ in range(world)]
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        for _ in range(2):  # pass 1 fills every rank's slot, pass 2 reduces complete data
            outs = [x.clone() for x in xs]
            for r in range(world):
                e.ar_allreduce(outs[r], bufs, r, cap, 2 * cap, 1, False, err)
        ref = sum(x.float() for x in xs)
        for r in range(world):
            torch.testing.assert_close(outs[r].float(), ref, rtol=1e-2 if dtype != torch.float32 else 1e-6, atol=1e-2)
            assert torch.equal(outs[r], outs[0])  # fixed summation order: identical on every rank
        assert int(err.item()) == 0
    finally:
        torch.cuda.synchronize()
        for b in bufs:
            e.ar_free(b)


def _two_procs_one_gpu():
    import torch.distributed as dist

    from scaling_amd.parallel.custom_allreduce import OneShotAllReduce

    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    rank = dist.get_rank()
    ar = OneShotAllReduce(dist.group.WORLD, torch.device("cuda", 0), capacity_bytes=4 << 20)
    assert ar.single_node
    for step, (n, dtype) in enumerate([(1024, torch.bfloat16), (65536, torch.float32), (8 * 1000, torch.float16),
                                       (1 << 20, torch.bfloat16)] * 3):
        g = torch.Generator(device="cuda").manual_seed(1000 * step + rank)
        x = torch.randn(n, device="cuda", dtype=dtype, generator=g)
        others = [torch.randn(n, device="cuda", dtype=dtype,
                              generator=torch.Generator(device="cuda").manual_seed(1000 * step + r))
                  for r in range(dist.get_world_size())]
        assert ar(x)
        ref = sum(o.float() for o in others)
        torch.testing.assert_close(x.float(), ref, rtol=1e-2, atol=2e-2)
    assert not ar(torch.zeros(8 << 20, device="cuda"))  # beyond capacity: caller falls back to RCCL
    ar.check()
    ar.close()
    dist.destroy_process_group()
    return True


def test_oneshot_allreduce_two_processes_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    assert all(run_distributed(_two_procs_one_gpu, 2, timeout=120).values())


def test_oneshot_timeout_poisons_output_and_sets_error():
    """A peer that never arrives: the bounded flag wait gives up, the output is NaN (not a sum of stale slots) and
    the error word is set (the optimizer raises on it at its per-step read)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    cap = 1 << 16
    e = _ext()
    own, other = e.ar_alloc(2 * cap + 256, 0)[0], e.ar_alloc(2 * cap + 256, 0)[0]
    try:
        x = torch.randn(4096, device="cuda", dtype=torch.bfloat16)
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        # rank 0 of a 2-rank group whose rank 1 ("other") never signals
        e.ar_allreduce(x, [own, other], 0, 0, 2 * cap, 7, True, err, 1 << 10)
        torch.cuda.synchronize()
        assert int(err.item()) == 1
        assert torch.isnan(x.float()).all()
    finally:
        torch.cuda.synchronize()
        e.ar_free(own)
        e.ar_free(other)
