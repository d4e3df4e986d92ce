"""Weight-gradient GEMM (ops.gemm.wgrad -> gemm_tn_ring_kernel) at the 7B layer shapes, T = 32768 tokens: TF/s per shape,
interleaved rounds.  Run under build variants (SCALING_AMD_EXT_SO) to A/B kernel changes.

usage: python tools/wgrad_bench.py [--rounds 3] [--iters 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops import gemm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--cold", type=int, default=1, help="operand sets rotated per call (4+: larger than the 256 MB MALL)")
a = ap.parse_args()
T = 32768
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008), "head": (32000, 4096)}
data = {}
for name, (n, k) in SHAPES.items():
    sets = [(torch.randn(T, n, device="cuda", dtype=torch.bfloat16), torch.randn(T, k, device="cuda", dtype=torch.bfloat16))
            for _ in range(a.cold)]
    out = torch.empty(n, k, device="cuda", dtype=torch.bfloat16)
    data[name] = (sets, out)
res = {k: [] for k in SHAPES}
for r in range(a.rounds):
    for name, (sets, out) in data.items():
        for i in range(2):
            gemm.wgrad(*sets[i % len(sets)], out)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(a.iters):
            gemm.wgrad(*sets[i % len(sets)], out)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.iters
        n, k = SHAPES[name]
        res[name].append(2 * T * n * k / ms / 1e9)
print(" ".join(f"{k} {max(v):.0f}" for k, v in res.items()), "TF (best of rounds)", flush=True)
