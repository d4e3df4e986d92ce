"""Stress test of the attention's bit-reproducibility next to another process's kernels (race forensics).

The 2-rank rehearsal occasionally gets a different attention backward for identical inputs (profiles/race_forensics_r5.md)
at a rate of ~1 in 30-200 calls.  This runs the RoPE-fused attention forward + backward ``--iters`` times against a
reference computed on an idle GPU and counts mismatching iterations while a second process loops one kind of kernel:

    none        nothing
    hip_wgrad   this framework's weight-gradient GEMM (gemm_tn_ring_kernel: LDS-DMA ring, transposing LDS reads)
    blas        a hipBLASLt GEMM (torch.matmul)
    attn        this framework's attention forward + backward
    bench       a whole llama_tiny training run (bench.py, one process)

    python tools/attn_stress.py --iters 2000 --hammer hip_wgrad
"""
from __future__ import annotations

import argparse
import json
import math
import os
import signal
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"race_tiny": (2, 256, 4, 2, 64), "d128": (2, 1024, 16, 4, 128)}


def hammer(kind: str, seconds: float) -> None:
    if kind == "bench":  # the full llama_tiny training step mix (norms, SwiGLU, GEMMs, attention, AdamW, copies)
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")}
        q = subprocess.Popen([sys.executable, os.path.join(root, "bench.py"), "--model", "llama_tiny", "--seq-len", "256",
                              "--micro-batch", "2", "--steps", "100000", "--warmup", "1"], cwd=root, env=env,
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        time.sleep(20)  # model build + first steps
        print("ready", flush=True)
        try:
            q.wait(timeout=seconds)
        except subprocess.TimeoutExpired:
            pass
        finally:
            q.kill()
            q.wait()
        return
    import torch

    from scaling_amd.ops import gemm

    dev = torch.device("cuda")
    if kind == "hip_wgrad":
        dy = torch.randn(512, 688, device=dev, dtype=torch.bfloat16)
        x = torch.randn(512, 256, device=dev, dtype=torch.bfloat16)
        dy2 = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16)
        x2 = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16)
        fns = [lambda: gemm.wgrad(dy, x), lambda: gemm.wgrad(dy2, x2)]
    elif kind == "blas":
        a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        fns = [lambda: torch.matmul(a, a)]
    elif kind == "attn":
        fns = [_attn_case(torch, "race_tiny")[0]]
    else:
        fns = []
    print("ready", flush=True)
    t0 = time.time()
    while time.time() - t0 < seconds:
        for f in fns:
            for _ in range(4):
                f()
        torch.cuda.synchronize()
        if not fns:
            time.sleep(0.01)


def _attn_case(torch, name):
    from scaling_amd.ops import attention, rope

    dev = torch.device("cuda")
    ns, S, HQ, HK, D = SHAPES[name]
    g = torch.Generator(device=dev).manual_seed(1)
    T = ns * S
    cu = torch.arange(0, T + 1, S, device=dev, dtype=torch.int32)
    base0 = torch.randn(T, (HQ + 2 * HK) * D, device=dev, dtype=torch.bfloat16, generator=g)
    do = torch.randn(T, HQ, D, device=dev, dtype=torch.bfloat16, generator=g)
    cos, sin = rope.rope_tables(D, S, 10000, False, torch.bfloat16, dev)
    pos = torch.arange(S, device=dev).repeat(ns)
    sc = 1 / math.sqrt(D)
    nq, nk = HQ * D, HK * D

    def run():
        base = base0.clone().requires_grad_(True)
        q = base[:, :nq].view(T, HQ, D)
        k = base[:, nq:nq + nk].view(T, HK, D)
        v = base[:, nq + nk:].view(T, HK, D)
        o = attention.rope_flash_attention(base, q, k, v, cos, sin, pos, D, S, False, cu, S, sc, True)
        o.backward(do)
        return o.detach(), base.grad

    return run, (HQ, HK, D, T)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--hammer", default="none", choices=["none", "hip_wgrad", "blas", "attn", "bench"])
    ap.add_argument("--shape", default="race_tiny", choices=sorted(SHAPES))
    ap.add_argument("--child", type=float, default=0.0)
    a = ap.parse_args()
    if a.child:
        hammer(a.hammer, a.child)
        return
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(1))  # a time limit still runs the finally below
    import torch

    run, (HQ, HK, D, T) = _attn_case(torch, a.shape)
    torch.cuda.synchronize()
    ref_o, ref_g = run()
    torch.cuda.synchronize()
    # own process group: the hammer and anything it starts (the bench hammer's training process) end together
    p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--hammer", a.hammer, "--child", "240"],
                         stdout=subprocess.PIPE, text=True, start_new_session=True)
    bad, bad_o, where = 0, 0, {}
    try:
        assert p.stdout is not None and p.stdout.readline().strip() == "ready"
        t0 = time.time()
        for it in range(a.iters):
            o, g = run()
            if not torch.equal(o, ref_o):
                bad_o += 1
            if not torch.equal(g, ref_g):
                bad += 1
                ne = (g != ref_g).reshape(T, -1)
                cols = torch.nonzero(ne.any(0)).reshape(-1)
                region = ["q" if c < HQ * D else ("k" if c < (HQ + HK) * D else "v") for c in cols.tolist()[:1]][0]
                where[region] = where.get(region, 0) + 1
                if bad <= 3:
                    print(json.dumps({"iter": it, "n": int(ne.sum()), "rows": torch.nonzero(ne.any(1)).reshape(-1)[:6].tolist(),
                                      "cols": cols[:8].tolist()}), flush=True)
            if time.time() - t0 > 200:
                break
    finally:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
    print(json.dumps({"shape": a.shape, "hammer": a.hammer, "iters": it + 1, "mismatch_grad": bad, "mismatch_out": bad_o,
                      "regions": where}), flush=True)


if __name__ == "__main__":
    main()
