"""Per-phase timing of the weight-gradient GEMM (s_memtime stamps of workgroup 0, 8 steady-state K-tiles).

Events per wave and K-tile: 0 loop top, 1 before the first barrier (reads + DMA + waits done), 2 after it,
3 MFMAs issued, 4 after the second barrier.  Prints per-group averages of the intervals (in s_memtime ticks).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (4096, 4096, 8192)))
ext().gemm_set_variant(int(os.environ.get("GEMM_VARIANT", "2")))
g = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    ext().gemm_tn(g, x, c, False)
for rep in range(3):
    d = ext().gemm_tn_timing(g, x, c).view(8, 8, 5).cpu().double()
    base = d[:, 0, 0].min()
    d = d - base
    print(f"rep {rep}")
    for w in range(8):
        rows = []
        for t in range(8):
            e = d[w, t]
            rows.append(f"[{e[0]:.0f} r{e[1]-e[0]:.0f} b{e[2]-e[1]:.0f} m{e[3]-e[2]:.0f} b{e[4]-e[3]:.0f}]")
        print(f"  wave {w}: " + " ".join(rows[:4]))
    per_tile = (d[:, 7, 4] - d[:, 0, 0]) / 7
    print("  ticks per K-tile per wave:", [round(float(v), 1) for v in per_tile])
    for grp in (0, 1):
        ws = list(range(4 * grp, 4 * grp + 4))
        sub = d[ws]
        r = (sub[:, :, 1] - sub[:, :, 0]).mean()
        b1 = (sub[:, :, 2] - sub[:, :, 1]).mean()
        m = (sub[:, :, 3] - sub[:, :, 2]).mean()
        b2 = (sub[:, :, 4] - sub[:, :, 3]).mean()
        if os.environ.get("GEMM_VARIANT", "2") == "6":
            print(f"  group {grp}: ksteps0-2 {r:.1f}  waits(lgkm+vm) {b1:.1f}  barrier {m:.1f}  kstep3+dma {b2:.1f}")
        else:
            print(f"  group {grp}: reads+dma {r:.1f}  barrier1 {b1:.1f}  mfma-issue {m:.1f}  barrier2 {b2:.1f}")
