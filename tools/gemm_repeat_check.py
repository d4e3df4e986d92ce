"""Determinism stress of the wgrad GEMM variants: the same product many times must be bit-identical and match fp32.

    python tools/gemm_repeat_check.py VARIANT [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

v = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
ext().gemm_set_variant(v)
bad = 0
for (M, N, K) in [(512, 768, 320), (512, 768, 384), (256, 512, 256), (6144, 4096, 8192), (1024, 512, 1024), (4096, 11008, 4096)]:
    torch.manual_seed(1)
    a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    ref = (a.float().t() @ b.float())
    c0 = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    ext().gemm_tn(a, b, c0, False)
    err = ((c0.float() - ref).abs().max() / ref.abs().max()).item()
    diffs = 0
    for _ in range(reps):
        c = torch.zeros_like(c0)
        ext().gemm_tn(a, b, c, False)
        diffs += int(not torch.equal(c, c0))
    print(f"variant {v} {M}x{N}x{K}: rel err {err:.4f}, runs differing from the first: {diffs}/{reps}", flush=True)
    bad += diffs + (err > 0.01)
print("REPEAT_OK" if bad == 0 else "REPEAT_FAIL")
