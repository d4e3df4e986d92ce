"""Weight-gradient layout probe at the 7B shapes: hand-written gemm_tn (dY^T X straight from token-major
operands) vs transposing dY once and running hipBLASLt in the dgrad-style layout (reduction-contiguous A).

    python tools/wgrad_layout_probe.py [--tokens 8192] [--iters 30]
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
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    T = a.tokens
    res = {}
    for name, (N, K) in SHAPES.items():
        g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        c = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        gT = g.t().contiguous()
        xT = x.t().contiguous()
        fl = 2 * T * N * K
        us = lambda f: timeit(f, a.iters) * 1e6  # noqa: E731
        r = {
            "ours_acc_us": us(lambda: ext().gemm_tn(g, x, c, True)),
            "blt_tn_acc_us": us(lambda: c.addmm_(g.t(), x)),
            "blt_gT_acc_us": us(lambda: c.addmm_(gT, x)),
            "blt_gT_xT_acc_us": us(lambda: c.addmm_(gT, xT.t())),
            "transpose_g_us": us(lambda: g.t().contiguous()),
            "transpose_x_us": us(lambda: x.t().contiguous()),
        }
        r["ours_tf"] = fl / r["ours_acc_us"] / 1e6
        r["blt_gT_tf"] = fl / r["blt_gT_acc_us"] / 1e6
        r["blt_gT_with_transpose_tf"] = fl / (r["blt_gT_acc_us"] + r["transpose_g_us"]) / 1e6
        r["blt_gT_xT_tf"] = fl / r["blt_gT_xT_acc_us"] / 1e6
        res[name] = {k: round(v, 1) for k, v in r.items()}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
