"""Weight-gradient GEMM at the 7B layer shapes: scaling_amd gemm_tn vs hipBLASLt (torch.matmul / addmm_).

    python tools/gemm_bench.py [--tokens 8192] [--iters 20]
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

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "mlp_in": (22016, 4096), "mlp_out": (4096, 11008), "head": (32000, 4096)}


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
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", type=str, default="", help="comma list of gemm_tn pipeline variants to compare")
    ap.add_argument("--rounds", type=int, default=5, help="interleaved timing rounds per variant (median reported)")
    a = ap.parse_args()
    T = a.tokens
    default_variant = ext().gemm_get_variant()
    out = {}
    for name, (Nout, Kin) in SHAPES.items():
        g = torch.randn(T, Nout, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, Kin, device="cuda", dtype=torch.bfloat16)
        c = torch.zeros(Nout, Kin, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * Nout * Kin
        ext().gemm_tn(g, x, c, False)
        ref = g.float().t() @ x.float()
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        c2 = c.clone()
        ext().gemm_tn(g, x, c2, True)
        err_acc = ((c2.float() - 2 * ref).abs().max() / ref.abs().max()).item()
        r = {}
        vs = [int(t) for t in a.variants.split(",") if t]
        for vv in vs:
            ext().gemm_set_variant(vv)
            cv = torch.zeros_like(c)
            ext().gemm_tn(g, x, cv, False)
            r[f"v{vv}_err"] = ((cv.float() - ref).abs().max() / ref.abs().max()).item()
            ca = c.clone()
            ext().gemm_tn(g, x, ca, True)
            r[f"v{vv}_err_acc"] = ((ca.float() - 2 * ref).abs().max() / ref.abs().max()).item()
        samples: dict = {vv: [] for vv in vs}
        for _ in range(a.rounds if vs else 0):  # interleaved rounds: variants see the same clock drift
            for vv in vs:
                ext().gemm_set_variant(vv)
                samples[vv].append(fl / timeit(lambda: ext().gemm_tn(g, x, c, True), a.iters) / 1e12)
        for vv in vs:
            r[f"v{vv}"] = sorted(samples[vv])[len(samples[vv]) // 2]
        ext().gemm_set_variant(default_variant)
        r.update({
            "ours": fl / timeit(lambda: ext().gemm_tn(g, x, c, False), a.iters) / 1e12,
            "ours_acc": fl / timeit(lambda: ext().gemm_tn(g, x, c, True), a.iters) / 1e12,
            "hipblaslt": fl / timeit(lambda: torch.matmul(g.t(), x), a.iters) / 1e12,
            "hipblaslt_addmm": fl / timeit(lambda: c.addmm_(g.t(), x), a.iters) / 1e12,
            "rel_err": err, "rel_err_acc": err_acc,
        })
        out[name] = r
        print(name, {k: round(v, 4 if "err" in k else 1) for k, v in r.items()}, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
