"""Decode GEMV micro-benchmark on one GPU: the 7B decode projections (q/k/v, o, gate/up, down) at batch 1 through
the plain, epilogue-fused and norm-prologue GEMV kernels; prints us per call and the weight-stream rate."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps: int = 200) -> float:
    for _ in range(10):
        fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / reps


def copies(shape, dev, dt, cold: bool):
    """Weight copies cycled through by the timed loop: > 1 GiB in total when cold, so every call streams its weight
    from HBM (the 256 MiB last-level cache holds a single 7B projection otherwise)."""
    nb = shape[0] * shape[1] * 2
    n = max(2, -(-(1 << 30) // nb)) if cold else 1
    return [torch.randn(*shape, device=dev, dtype=dt) / 64 for _ in range(n)]


def main() -> None:
    from scaling_amd.ops._ext import ext
    from scaling_amd.ops import norm as norm_ops

    torch.manual_seed(0)
    dev, dt = "cuda", torch.bfloat16
    H, F, M = 4096, 11008, int(os.environ.get("ROWS", "1"))
    x = torch.randn(M, H, device=dev, dtype=dt)
    add = torch.randn(M, H, device=dev, dtype=dt)
    g = torch.ones(H, device=dev, dtype=dt)
    cold = os.environ.get("COLD", "1") != "0"
    wqkv = copies((3 * H, H), dev, dt, cold)
    wo = copies((H, H), dev, dt, cold)
    wgu = copies((2 * F, H), dev, dt, cold)
    wd = copies((H, F), dev, dt, cold)
    a = torch.randn(M, F, device=dev, dtype=dt)
    W = lambda ws, i: ws[i % len(ws)]  # noqa: E731
    cases = [
        ("norm_row (rmsnorm, 1 launch)", lambda i: norm_ops.add_rms_norm(x, add, g, 1e-5), None),
        ("qkv gemv", lambda i: ext().gemv(x, W(wqkv, i), None), wqkv),
        ("qkv gemv_norm", lambda i: ext().gemv_norm(x, None, g, 1e-5, W(wqkv, i), 0), wqkv),
        ("o gemv_residual", lambda i: ext().gemv_residual(x, W(wo, i), add), wo),
        ("gate/up gemv (plain, 2F rows)", lambda i: ext().gemv(x, W(wgu, i), None), wgu),
        ("gate/up gemv_swiglu", lambda i: ext().gemv_swiglu(x, W(wgu, i)), wgu),
        ("gate/up gemv_norm swiglu", lambda i: ext().gemv_norm(x, add, g, 1e-5, W(wgu, i), 2), wgu),
        ("down gemv_residual", lambda i: ext().gemv_residual(a, W(wd, i), add), wd),
    ]
    print(f"rows {M}, {'cold (weights cycled through > 1 GiB)' if cold else 'warm (one weight copy)'}", flush=True)
    for name, fn, w in cases:
        us = timeit(fn)
        nb = w[0].numel() * w[0].element_size() if w is not None else 0
        print(f"{name:34s} {us:8.2f} us  {nb / us / 1e6 if nb else 0:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
