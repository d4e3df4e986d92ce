"""The rehearsal's host-staged collectives (scaling_amd/core/topology/gloo_gpu.py) return what the plain gloo
collectives return (here on CPU ranks, with the device-tensor test forced on so the staging path runs)."""
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from scaling_amd.core.utils.port import find_free_port


def _worker(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from scaling_amd.core.topology import gloo_gpu

    gloo_gpu._cuda = lambda t: isinstance(t, torch.Tensor)  # every tensor takes the staged path
    gloo_gpu.install()
    x = torch.arange(8, dtype=torch.float32) + 10 * rank
    a = x.clone()
    w = dist.all_reduce(a, async_op=True)
    assert w.wait()
    rs = torch.empty(8 // world)
    dist.reduce_scatter_tensor(rs, x.clone())
    ag = torch.empty(8 * world)
    dist.all_gather_into_tensor(ag, x[:8:1].clone())
    bc = x.clone()
    dist.broadcast(bc, src=1)
    lst = [torch.empty(8) for _ in range(world)]
    dist.all_gather(lst, x)
    # plain lists: a tensor on the queue travels by file descriptor, which dies with this process
    q.put((rank, a.tolist(), rs.tolist(), ag.tolist(), bc.tolist(), torch.stack(lst).tolist()))
    dist.destroy_process_group()


import pytest


@pytest.mark.parametrize("world", [2, 4])
def test_host_staged_collectives_match_gloo(world):
    port = find_free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    xs = [torch.arange(8, dtype=torch.float32) + 10 * r for r in range(world)]
    tot = sum(xs[1:], xs[0].clone())
    per = 8 // world
    for r in range(world):
        a, rs, ag, bc, lst = (torch.tensor(v) for v in res[r])
        assert torch.equal(a, tot)
        assert torch.equal(rs, tot[per * r: per * (r + 1)])
        assert torch.equal(ag, torch.cat(xs))
        assert torch.equal(bc, xs[1])
        assert torch.equal(lst, torch.stack(xs))


def _async_worker(rank: int, world: int, port: int, q) -> None:
    """Asynchronous rehearsal mode, host side: the C++ worker (csrc/rehearsal.cpp) runs queued collectives on the
    group's ProcessGroup in program order and opens each job's gate word; Python-level gloo calls (CPU tensors, objects,
    barrier) take their turn between them.  Here the gate words are a CPU tensor and the jobs have no event."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from scaling_amd.core.topology import gloo_gpu
    from scaling_amd.ops._ext import ext

    gloo_gpu._ASYNC = True
    gloo_gpu.install()
    x = torch.arange(8, dtype=torch.float32) + 10 * rank
    flags = torch.zeros(64, dtype=torch.int32)
    pg = dist.distributed_c10d._get_default_group()
    hs = []
    for i in range(20):  # C++ jobs interleaved with Python-level calls: any reordering would mismatch the ranks
        h = x.clone() * (i + 1)
        ext().rw_collective(0, pg, h, h, 0, 0, 0, flags.data_ptr(), i, 1)  # all_reduce SUM, gate word i
        hs.append(h)
        a = x.clone() * (i + 1)
        dist.all_reduce(a)  # Python-level gloo call in its turn
    g = torch.empty(8 * world)
    ext().rw_collective(3, pg, x.clone(), g, 0, 0, 0, flags.data_ptr(), 20, 1)  # all_gather_into
    m = x.clone()
    ext().rw_collective(0, pg, m, m, 1, 0, 0, flags.data_ptr(), 21, 1)  # all_reduce MAX
    objs = [None] * world
    dist.all_gather_object(objs, {"rank": rank})
    dist.barrier()
    ext().rw_drain()
    ext().rw_check()
    t0 = time.time()
    while int(flags[:22].min()) < 1 and time.time() - t0 < 30:
        time.sleep(0.01)
    q.put((rank, [h.tolist() for h in hs], g.tolist(), m.tolist(), [o["rank"] for o in objs], flags[:22].tolist()))
    dist.destroy_process_group()


def test_async_mode_worker_orders_jobs_and_host_calls():
    world = 2
    port = find_free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_async_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    xs = [torch.arange(8, dtype=torch.float32) + 10 * r for r in range(world)]
    tot = sum(xs[1:], xs[0].clone())
    for r in range(world):
        hs, g, m, ranks, flags = res[r]
        assert all(torch.equal(torch.tensor(h), tot * (i + 1)) for i, h in enumerate(hs))
        assert torch.equal(torch.tensor(g), torch.cat(xs))
        assert torch.equal(torch.tensor(m), torch.maximum(xs[0], xs[1]))
        assert ranks == list(range(world)) and flags == [1] * 22


def _async_p2p_worker(rank: int, world: int, port: int, q) -> None:
    """Asynchronous rehearsal p2p, host side: send jobs POST their gloo sends without waiting (both ranks send first,
    then receive -- a worker that waited for its sends would deadlock here), receive jobs open their gate once the data
    arrived, and ``rw_send_wait`` inside a host turn retires a send batch."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from scaling_amd.ops._ext import ext

    pg = dist.distributed_c10d._get_default_group()
    flags = torch.zeros(8, dtype=torch.int32)
    peer = 1 - rank
    outs = []
    for i in range(3):
        payload = [torch.full((5,), float(10 * rank + i)), torch.arange(3, dtype=torch.int64) + rank]
        ext().rw_p2p_send(pg, payload, [peer, peer], [0, 0], 0, i)
        got = [torch.empty(5), torch.empty(3, dtype=torch.int64)]
        ext().rw_p2p_recv(pg, got, [peer, peer], [0, 0], flags.data_ptr(), i, 1)
        outs.append(got)
    t = ext().rw_host_begin()
    for i in range(3):
        ext().rw_send_wait(i)
    ext().rw_host_end(t)
    ext().rw_drain()
    ext().rw_check()
    t0 = time.time()
    while int(flags[:3].min()) < 1 and time.time() - t0 < 30:
        time.sleep(0.01)
    q.put((rank, [[a.tolist(), b.tolist()] for a, b in outs], flags[:3].tolist()))
    dist.destroy_process_group()


def test_async_mode_worker_p2p_posts_sends():
    world = 2
    port = find_free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_async_p2p_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        outs, flags = res[r]
        peer = 1 - r
        assert flags == [1, 1, 1]
        for i, (a, b) in enumerate(outs):
            assert a == [float(10 * peer + i)] * 5 and b == [peer, peer + 1, peer + 2]
