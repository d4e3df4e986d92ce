"""Run one weight-gradient GEMM shape repeatedly (for rocprofv3 counter collection)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (4096, 4096, 8192)))
which = sys.argv[4] if len(sys.argv) > 4 else "ours"
g = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(10):
    if which == "ours":
        ext().gemm_tn(g, x, c, False)
    else:
        torch.matmul(g.t(), x, out=c)
torch.cuda.synchronize()
