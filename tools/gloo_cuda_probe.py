"""Which torch.distributed collectives does the gloo backend accept for GPU tensors?

Runs 2 ranks on one GPU (RCCL refuses two ranks per device, gloo does not) and tries every collective the
framework issues (optimizer, TP regions, pipe p2p, data broadcast) with ``cuda`` tensors, on the default and
on a side stream.  Decides whether a multi-rank rehearsal on a 1-GPU box can run the GPU code paths with
gloo standing in for RCCL.  Usage: ``python tools/gloo_cuda_probe.py`` (spawns its own ranks).
"""
import json
import os
import subprocess
import sys


def worker() -> None:
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    res = {}

    def attempt(name, fn):
        try:
            ok = fn()
            torch.cuda.synchronize()
            res[name] = "ok" if ok in (None, True) else f"wrong:{ok}"
        except Exception as e:  # noqa: BLE001
            res[name] = f"err:{type(e).__name__}:{str(e)[:120]}"

    def ar():
        x = torch.full((1000,), float(rank + 1), device=dev)
        dist.all_reduce(x)
        return bool((x == 3).all().item())

    def rs():
        x = torch.arange(8, dtype=torch.float32, device=dev) + rank
        out = torch.empty(4, device=dev)
        dist.reduce_scatter_tensor(out, x)
        exp = (torch.arange(8, dtype=torch.float32) * 2 + 1)[rank * 4:(rank + 1) * 4]
        return bool(torch.equal(out.cpu(), exp))

    def rs_bf16():
        x = (torch.arange(8, dtype=torch.float32, device=dev) + rank).bfloat16()
        out = torch.empty(4, device=dev, dtype=torch.bfloat16)
        dist.reduce_scatter_tensor(out, x)
        return True

    def ag():
        x = torch.full((4,), float(rank), device=dev, dtype=torch.bfloat16)
        out = torch.empty(8, device=dev, dtype=torch.bfloat16)
        dist.all_gather_into_tensor(out, x)
        return bool(out[4:].eq(1).all().item() and out[:4].eq(0).all().item())

    def ag_list():
        x = torch.full((4,), float(rank), device=dev, dtype=torch.float64)
        outs = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(outs, x)
        return bool(outs[1].eq(1).all().item())

    def bc():
        x = torch.full((16,), float(rank), device=dev)
        dist.broadcast(x, src=0)
        return bool(x.eq(0).all().item())

    def p2p():
        x = torch.full((16,), float(rank), device=dev)
        y = torch.empty(16, device=dev)
        peer = 1 - rank
        ops = [dist.P2POp(dist.isend, x, peer), dist.P2POp(dist.irecv, y, peer)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        return bool(y.eq(peer).all().item())

    def sendrecv():
        x = torch.full((16,), float(rank), device=dev)
        if rank == 0:
            dist.send(x, 1)
        else:
            dist.recv(x, 0)
        return bool(x.eq(0).all().item())

    def side_stream_ar():
        s = torch.cuda.Stream()
        x = torch.full((1 << 20,), float(rank + 1), device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            dist.all_reduce(x)
            ev = torch.cuda.Event()
            ev.record(s)
        torch.cuda.current_stream().wait_event(ev)
        return bool((x == 3).all().item())

    def async_ag():
        x = torch.full((4,), float(rank), device=dev)
        out = torch.empty(8, device=dev)
        w = dist.all_gather_into_tensor(out, x, async_op=True)
        w.wait()
        return bool(out[4:].eq(1).all().item())

    for n, f in [("all_reduce", ar), ("reduce_scatter_tensor", rs), ("reduce_scatter_tensor_bf16", rs_bf16),
                 ("all_gather_into_tensor", ag), ("all_gather", ag_list), ("broadcast", bc),
                 ("batch_isend_irecv", p2p), ("send_recv", sendrecv), ("side_stream_all_reduce", side_stream_ar),
                 ("async_all_gather_into_tensor", async_ag)]:
        attempt(n, f)
        dist.barrier()
    if rank == 0:
        print(json.dumps(res, indent=1), flush=True)
    dist.destroy_process_group()


def main() -> int:
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT="29655", GLOO_PROBE_WORKER="1")
    procs = [subprocess.Popen([sys.executable, __file__], env=dict(env, RANK=str(r))) for r in range(2)]
    codes = [p.wait(timeout=300) for p in procs]
    return max(abs(c) for c in codes)


if __name__ == "__main__":
    if os.environ.get("GLOO_PROBE_WORKER"):
        worker()
    else:
        sys.exit(main())
