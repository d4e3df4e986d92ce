"""Per-k-step s_memtime stamps of the forward GEMM ring kernel (gemm_nt), workgroup 0, k-steps 32-39: events 0 top,
1 MFMA stream issued, 2 reads retired, 3 pieces landed, 4 past the barrier.

    python tools/gemm_nt_timing.py [M N K]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (32768, 4096, 4096)))
a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    ext().gemm_nt(a, b, c, False)
for rep in range(3):
    d = ext().gemm_nt_timing(a, b, c).view(4, 8, 5).cpu().double()
    d = d - d[:, 0, 0].min()
    per = (d[:, 7, 4] - d[:, 0, 0]) / 8
    names = ["mfma-stream", "lgkm-wait", "vm-wait", "barrier"]
    print(f"rep {rep} cycles per k-step per wave:", [round(float(v), 1) for v in per],
          {n: round(float((d[:, :, e + 1] - d[:, :, e]).mean()), 1) for e, n in enumerate(names)})
