"""Is the flash attention (forward + backward) bitwise reproducible while other work runs on the GPU?

The race check (tests/test_gpu_rehearsal.py) runs several ranks on one GPU; a kernel whose result depends on which
waves run when (an unsynchronised LDS hand-off, a missing wait) gives different bits only under such load.  This
runs the attention alone: the reference result on an idle GPU, then trials (a) idle, (b) with a big GEMM queued on a
second stream of this process, (c) while another process hammers the GPU with GEMMs, and counts the trials whose
o / dq / dk / dv differ from the reference in any bit.

    python tools/attn_repro.py [--trials 20]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (n_seq, seq, Hq, Hkv, D)
    "race_tiny": (2, 256, 4, 2, 64),
    "race_tiny_r256_docs": (4, 128, 4, 2, 64),
    "7b_s4096": (2, 4096, 32, 8, 128),
}


def hammer(seconds: float) -> None:
    import torch

    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    print("ready", flush=True)
    t0 = time.time()
    while time.time() - t0 < seconds:
        for _ in range(8):
            torch.matmul(a, b)
        torch.cuda.synchronize()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    ap.add_argument("--hammer", type=float, default=0.0)
    a = ap.parse_args()
    if a.hammer:
        hammer(a.hammer)
        return
    import torch

    from scaling_amd.ops import attention, rope

    dev = torch.device("cuda")
    side = torch.cuda.Stream()
    big = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for name, (ns, S, HQ, HK, D) in SHAPES.items():
        g = torch.Generator(device=dev).manual_seed(1)
        T = ns * S
        cu = torch.arange(0, T + 1, S, device=dev, dtype=torch.int32)
        q0 = torch.randn(T, HQ, D, device=dev, dtype=torch.bfloat16, generator=g)
        k0 = torch.randn(T, HK, D, device=dev, dtype=torch.bfloat16, generator=g)
        v0 = torch.randn(T, HK, D, device=dev, dtype=torch.bfloat16, generator=g)
        do = torch.randn(T, HQ, D, device=dev, dtype=torch.bfloat16, generator=g)
        sc = 1 / math.sqrt(D)

        cos, sin = rope.rope_tables(D, S, 10000, False, torch.bfloat16, dev)
        pos = torch.arange(S, device=dev).repeat(ns)
        base0 = torch.cat([q0.reshape(T, -1), k0.reshape(T, -1), v0.reshape(T, -1)], dim=1)

        def run_plain():
            q, k, v = (t.clone().requires_grad_(True) for t in (q0, k0, v0))
            o = attention.flash_attention(q, k, v, cu, cu, S, S, sc, True, None)
            o.backward(do)
            return [o.detach(), q.grad, k.grad, v.grad]

        def run_rope():  # the training path: RoPE fused into the attention (inverse rotation in the dQ/dK epilogues)
            base = base0.clone().requires_grad_(True)
            nq, nk = HQ * D, HK * D
            q = base[:, :nq].view(T, HQ, D)
            k = base[:, nq:nq + nk].view(T, HK, D)
            v = base[:, nq + nk:].view(T, HK, D)
            o = attention.rope_flash_attention(base, q, k, v, cos, sin, pos, D, S, False, cu, S, sc, True)
            assert o is not None, "fused rope + flash path declined"
            o.backward(do)
            g = base.grad
            return [o.detach(), g[:, :nq], g[:, nq:nq + nk], g[:, nq + nk:]]

        run = run_rope if os.environ.get("ATTN_REPRO_ROPE", "1") == "1" else run_plain

        torch.cuda.synchronize()
        ref = run()
        torch.cuda.synchronize()
        names = ["o", "dq", "dk", "dv"]

        def count(out, res):
            for n, x, y in zip(names, out, ref):
                res[n] += int(not torch.equal(x, y))

        res = {c: {n: 0 for n in names} for c in ("idle", "side_stream", "other_process")}
        for _ in range(a.trials):
            count(run(), res["idle"])
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                for _ in range(2):
                    torch.matmul(big, big)
            out = run()  # runs while the side stream's GEMMs occupy part of the chip
            torch.cuda.synchronize()
            count(out, res["side_stream"])
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--hammer", "60"], stdout=subprocess.PIPE,
                             text=True)
        try:
            assert p.stdout is not None and p.stdout.readline().strip() == "ready"
            for _ in range(a.trials):
                count(run(), res["other_process"])
                torch.cuda.synchronize()
        finally:
            p.kill()
            p.wait()
        print(json.dumps({"shape": name, "trials": a.trials, **res}), flush=True)


if __name__ == "__main__":
    main()
