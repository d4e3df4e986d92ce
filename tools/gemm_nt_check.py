"""Correctness sweep of the NT GEMM kernel (csrc/kernels/gemm_nt.hip) against an fp32 reference: small to 7B shapes,
and a per-64-deep-stage probe (all other k-stages zeroed) that localises a pipeline error to a stage."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402


def err(M, N, K, x=None, w=None):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) if x is None else x
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) if w is None else w
    c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    ext().gemm_nt(x, w, c)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t()
    d = (c.float() - ref).abs()
    bad = (d > 0.02 * ref.abs().max()).float()
    return (d.max() / ref.abs().max()).item(), bad.mean().item(), bad


# the last three have more tiles than CUs: persistent workgroups walk 1-3 tiles each
for (M, N, K) in [(256, 256, 256), (256, 256, 1024), (256, 256, 4096), (512, 512, 4096), (2048, 2048, 4096),
                  (4096, 4096, 4096), (8192, 2304, 256), (4352, 4096, 384), (4096, 8448, 512)]:
    e, frac, bad = err(M, N, K)
    msg = f"M{M} N{N} K{K}: max_rel_err {e:.4f} bad_frac {frac:.4f}"
    if frac > 0:
        rows = bad.sum(1).nonzero().flatten()
        cols = bad.sum(0).nonzero().flatten()
        msg += (f" bad rows%256 {sorted(set((rows % 256).tolist()))[:16]}"
                f" bad cols%256 {sorted(set((cols % 256).tolist()))[:16]}")
    print(msg, flush=True)
M, N, K = 256, 256, 1024
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
for s in range(K // 64):
    xs = torch.zeros_like(x)
    xs[:, 64 * s:64 * s + 64] = x[:, 64 * s:64 * s + 64]
    e, frac, _ = err(M, N, K, xs, w)
    print(f"stage {s}: max_rel_err {e:.4f} bad_frac {frac:.4f}", flush=True)
