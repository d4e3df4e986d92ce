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
    """Asynchronous rehearsal mode, host side: every gloo call (CPU tensors, objects, barrier) runs on the one worker
    thread in program order and returns what plain gloo returns."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from scaling_amd.core.topology import gloo_gpu

    gloo_gpu._ASYNC = True
    gloo_gpu.install()
    x = torch.arange(8, dtype=torch.float32) + 10 * rank
    outs = []
    for i in range(20):  # many small calls back to back: any cross-thread reordering would mismatch the ranks
        a = x.clone() * (i + 1)
        dist.all_reduce(a)
        outs.append(a.tolist())
    objs = [None] * world
    dist.all_gather_object(objs, {"rank": rank})
    dist.barrier()
    q.put((rank, outs, [o["rank"] for o in objs], gloo_gpu._state["worker"].t.name))
    dist.destroy_process_group()


def test_async_mode_host_calls_through_one_worker():
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
    tot = sum((torch.arange(8, dtype=torch.float32) + 10 * r for r in range(world)))
    for r in range(world):
        outs, ranks, tname = res[r]
        assert all(torch.equal(torch.tensor(o), tot * (i + 1)) for i, o in enumerate(outs))
        assert ranks == list(range(world)) and tname == "gloo-gpu-async"
