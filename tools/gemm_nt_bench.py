"""Forward / input-gradient GEMM at the 7B layer shapes: scaling_amd gemm_nt (C = A B^T, HIP ring kernel) vs hipBLASLt
(torch.nn.functional.linear with the repo's TunableOp table, as the training step runs it).

    python tools/gemm_nt_bench.py [--tokens 32768] [--iters 10]
Prints TF/s per shape and the max error against an fp32 reference.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

# name: (N out, K in) of y = x W^T; dgrad shapes are the same products with N and K swapped (x = dY, W^T cached)
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "mlp_in": (22016, 4096), "mlp_out": (4096, 11008),
          "head": (32000, 4096), "dgrad_qkv": (4096, 6144), "dgrad_mlp_in": (4096, 22016), "dgrad_mlp_out": (11008, 4096)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tuned", type=int, default=1, help="use the repo's TunableOp table for hipBLASLt")
    a = ap.parse_args()
    if a.tuned:
        from scaling_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms("use", None, 0)
    T = a.tokens
    out = {}
    for name, (N, K) in SHAPES.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        c = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * N * K
        ok = ext().gemm_nt_ok(x, w, c)
        r = {}
        if ok:
            ext().gemm_nt(x, w, c, False)
            ref = x[:2048].float() @ w.float().t()
            r["rel_err"] = ((c[:2048].float() - ref).abs().max() / ref.abs().max()).item()
        ours, blas = [], []
        for _ in range(a.rounds):
            if ok:
                ours.append(fl / timeit(lambda: ext().gemm_nt(x, w, c, False), a.iters) / 1e12)
            blas.append(fl / timeit(lambda: torch.nn.functional.linear(x, w), a.iters) / 1e12)
        if ours:
            r["ours"] = sorted(ours)[len(ours) // 2]
        r["hipblaslt"] = sorted(blas)[len(blas) // 2]
        out[name] = r
        print(name, {k: round(v, 4 if "err" in k else 1) for k, v in r.items()}, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
