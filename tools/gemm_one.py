"""Runs the weight-gradient GEMM at one shape a few times (a short program for rocprofv3 --pmc passes).

    python tools/gemm_one.py M N K [iters]      (GEMM_VARIANT env selects the pipeline variant)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
ext().gemm_set_variant(int(os.environ.get("GEMM_VARIANT", "2")))
g = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    ext().gemm_tn(g, x, c, True)
torch.cuda.synchronize()
print("done", M, N, K, iters)
