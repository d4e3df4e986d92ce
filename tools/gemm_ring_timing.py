"""Per-k-step timing of the ring wgrad GEMM (variants 9-12): s_memtime stamps of workgroup 0, k-steps 32-39.

Events per wave and k-step: 0 top, 1 MFMA stream issued (reads + pieces threaded in), 2 reads retired (lgkmcnt 0),
3 pieces landed (vmcnt), 4 past the barrier.  Prints per-wave intervals and their means (s_memtime ticks = cycles).

    GEMM_VARIANT=10 python tools/gemm_ring_timing.py [M N K]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (4096, 4096, 16384)))
ext().gemm_set_variant(int(os.environ.get("GEMM_VARIANT", "10")))
g = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    ext().gemm_tn(g, x, c, False)
for rep in range(3):
    d = ext().gemm_tn_timing(g, x, c)[:160].view(4, 8, 5).cpu().double()
    d = d - d[:, 0, 0].min()
    print(f"rep {rep}")
    for w in range(4):
        rows = [f"[m{d[w, t, 1] - d[w, t, 0]:.0f} l{d[w, t, 2] - d[w, t, 1]:.0f} v{d[w, t, 3] - d[w, t, 2]:.0f} "
                f"b{d[w, t, 4] - d[w, t, 3]:.0f}]" for t in range(4)]
        print(f"  wave {w}: " + " ".join(rows))
    per = (d[:, 7, 4] - d[:, 0, 0]) / 8
    print("  cycles per k-step per wave:", [round(float(v), 1) for v in per], " (64 MFMAs x 16 = 1024 ideal)")
    names = ["mfma-stream", "lgkm-wait", "vm-wait", "barrier"]
    print("  means:", {n: round(float((d[:, :, e + 1] - d[:, :, e]).mean()), 1) for e, n in enumerate(names)})
