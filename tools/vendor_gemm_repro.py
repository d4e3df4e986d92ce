"""Standalone reproducer (torch only, none of this framework's code or streams): does a vendor GEMM (hipBLASLt by
default on gfx950, rocBLAS with TORCH_BLAS_PREFER_HIPBLASLT=0) return bitwise-different results for the same inputs
when another stream's kernel is running on the GPU at the same time?

    python tools/vendor_gemm_repro.py [--trials 20]

Shapes: the GEMMs of the llama_tiny race-check model (h 256, ffn 688, 512 tokens per rank) that the framework sends to
the vendor library (weight gradients whose M / N are not multiples of 256 before round 5, and the forward / dgrad
GEMMs).  For each shape the result on an idle GPU is the reference; then every trial recomputes it (a) on the idle GPU
and (b) right after a large bf16 GEMM was queued on a second stream (the two run concurrently), and counts the trials
whose result differs from the reference in any bit.  Each environment variant runs in a fresh process.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys


def worker(trials: int) -> None:
    import torch

    if os.environ.get("REPRO_DETERMINISTIC") == "1":
        torch.use_deterministic_algorithms(True)
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape):
        return torch.randn(*shape, device=dev, dtype=torch.bfloat16, generator=g)

    T = 512
    cases = []
    # (name, fn) -- fn() computes into a fresh / fixed output and returns it
    for n_out, k_in in ((1376, 256), (256, 688), (512, 256), (256, 256)):
        dy, x = rnd(T, n_out), rnd(T, k_in)
        flat = torch.zeros(n_out * k_in + 4096, device=dev, dtype=torch.bfloat16)
        view = flat[1024 : 1024 + n_out * k_in].view(n_out, k_in)  # a gradient view inside a flat buffer
        base = rnd(n_out, k_in)

        def wgrad_out(dy=dy, x=x, view=view):
            torch.matmul(dy.t(), x, out=view)
            return view.clone()

        def wgrad_acc(dy=dy, x=x, view=view, base=base):
            view.copy_(base)
            view.addmm_(dy.t(), x)
            return view.clone()

        cases.append((f"wgrad out= [{n_out},{k_in}] T{T}", wgrad_out))
        cases.append((f"wgrad addmm_ [{n_out},{k_in}] T{T}", wgrad_acc))
        w = rnd(n_out, k_in)
        xin = rnd(T, k_in)
        cases.append((f"fwd x W^T [{T},{k_in}]x[{n_out},{k_in}]^T", lambda xin=xin, w=w: torch.nn.functional.linear(xin, w)))
        gy = rnd(T, n_out)
        cases.append((f"dgrad dY W [{T},{n_out}]x[{n_out},{k_in}]", lambda gy=gy, w=w: torch.matmul(gy, w)))

    side = torch.cuda.Stream()
    big_a, big_b = rnd(8192, 8192), rnd(8192, 8192)
    mid_a, mid_b = rnd(2048, 4096), rnd(4096, 2048)
    out = []
    for name, fn in cases:
        torch.cuda.synchronize()
        ref = fn()
        torch.cuda.synchronize()
        res = {"case": name, "idle_diff": 0, "busy_big_diff": 0, "busy_mid_diff": 0, "trials": trials}
        for _ in range(trials):
            torch.cuda.synchronize()
            r = fn()
            torch.cuda.synchronize()
            res["idle_diff"] += int(not torch.equal(r, ref))
            for tag, (a, b) in (("busy_big_diff", (big_a, big_b)), ("busy_mid_diff", (mid_a, mid_b))):
                torch.cuda.synchronize()
                with torch.cuda.stream(side):
                    torch.matmul(a, b)
                r = fn()  # queued right behind the side stream's GEMM: runs concurrently with it
                torch.cuda.synchronize()
                res[tag] += int(not torch.equal(r, ref))
        out.append(res)
        print(json.dumps(res), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    ap.add_argument("--worker", action="store_true")
    a = ap.parse_args()
    if a.worker:
        worker(a.trials)
        return
    variants = [
        ("hipblaslt-default", {}),
        ("hipblaslt-deterministic", {"REPRO_DETERMINISTIC": "1", "ROCBLAS_DEFAULT_ATOMICS_MODE": "0",
                                     "CUBLAS_WORKSPACE_CONFIG": ":4096:8"}),
        ("rocblas-deterministic", {"REPRO_DETERMINISTIC": "1", "ROCBLAS_DEFAULT_ATOMICS_MODE": "0",
                                   "CUBLAS_WORKSPACE_CONFIG": ":4096:8", "TORCH_BLAS_PREFER_HIPBLASLT": "0"}),
    ]
    for tag, env in variants:
        print(f"== {tag} {env}", flush=True)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", "--trials", str(a.trials)],
                           env={**os.environ, **env}, timeout=600)
        if r.returncode != 0:
            raise SystemExit(r.returncode)


if __name__ == "__main__":
    main()
