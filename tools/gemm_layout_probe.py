"""Weight-gradient GEMM layout probe at the 7B bench shapes (T tokens):

    dW[Nout, Kin] = dY^T X,   dY: [T, Nout], X: [T, Kin]  (both token-major, the reduction runs over T)

Times (TFLOP/s): the hand-written TN kernel (gemm_tn), hipBLASLt on the same TN layout, hipBLASLt with dY
transposed once ("NN": dY^T contiguous), with both transposed ("NT": both operands k-contiguous), and the
transpose2d cost of each operand.  Answers whether materialising k-contiguous copies pays.

    python tools/gemm_layout_probe.py [--tokens 32768] [--iters 10]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "mlp_in": (22016, 4096), "mlp_out": (4096, 11008)}


def timeit(fn, iters):
    for _ in range(2):
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
    ap.add_argument("--tune", action="store_true", help="TunableOp-tune the hipBLASLt layouts first (as the bench does)")
    a = ap.parse_args()
    if a.tune:
        from scaling_amd.utils.gemm_tuning import enable_tuned_gemms

        print("gemm tuning:", enable_tuned_gemms("tune", "/tmp/gemm_layout_probe_tuned.csv"), flush=True)
    T = a.tokens
    out = {}
    tot = {"ours": 0.0, "tn": 0.0, "nn": 0.0, "nt": 0.0, "tr_dy": 0.0, "tr_x": 0.0}
    for name, (Nout, Kin) in SHAPES.items():
        g = torch.randn(T, Nout, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, Kin, device="cuda", dtype=torch.bfloat16)
        c = torch.zeros(Nout, Kin, device="cuda", dtype=torch.bfloat16)
        gT = ext().transpose2d(g)
        xT = ext().transpose2d(x)
        fl = 2 * T * Nout * Kin
        r = {
            "ours": timeit(lambda: ext().gemm_tn(g, x, c, True), a.iters),
            "tn": timeit(lambda: c.addmm_(g.t(), x), a.iters),
            "nn": timeit(lambda: c.addmm_(gT, x), a.iters),
            "nt": timeit(lambda: c.addmm_(gT, xT.t()), a.iters),
            "tr_dy": timeit(lambda: ext().transpose2d(g), a.iters),
            "tr_x": timeit(lambda: ext().transpose2d(x), a.iters),
        }
        for k in tot:
            tot[k] += r[k]
        row = {k: (round(fl / v / 1e12, 1) if not k.startswith("tr") else round(v * 1e3, 3)) for k, v in r.items()}
        row["ms"] = {k: round(v * 1e3, 3) for k, v in r.items()}
        out[name] = row
        print(name, "TF/s:", {k: v for k, v in row.items() if k != "ms"}, "ms:", row["ms"], flush=True)
        del g, x, c, gT, xT
        torch.cuda.empty_cache()
    per_layer = {k: round(v * 1e3, 3) for k, v in tot.items()}
    print("per layer ms:", per_layer, "x32 layers:", {k: round(v * 32, 1) for k, v in per_layer.items()})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
