"""Runs the forward GEMM kernel (gemm_nt) at one shape a few times (a short program for rocprofv3 --pmc).

    python tools/gemm_nt_one.py M N K [iters]
"""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    ext().gemm_nt(a, b, c)
torch.cuda.synchronize()
print("done", M, N, K, iters)
