"""Forward / input-gradient GEMM at the 7B layer shapes: scaling_amd gemm_nt (C = A B^T, csrc/kernels/gemm_nt.hip) vs
hipBLASLt (torch.nn.functional.linear with the repo's TunableOp table, as the training step runs it), plus the fused
SwiGLU epilogues against hipBLASLt + the stand-alone SwiGLU kernels.

    python tools/gemm_nt_bench.py [--tokens 32768] [--iters 10] [--rounds 3]
Prints TF/s per shape (median over rounds, interleaved) and the max error against an fp32 reference.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

# name: (N out, K in) of y = x W^T; dgrad shapes are the same products with N and K swapped (x = dY, W^T cached)
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "mlp_in": (22016, 4096), "mlp_out": (4096, 11008),
          "head": (32000, 4096), "dgrad_qkv": (4096, 6144), "dgrad_mlp_in": (4096, 22016), "dgrad_mlp_out": (11008, 4096)}


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def med(x):
    return sorted(x)[len(x) // 2]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tuned", type=int, default=1, help="use the repo's TunableOp table for hipBLASLt")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    if a.tuned:
        from scaling_amd.utils.gemm_tuning import enable_tuned_gemms
        enable_tuned_gemms("use", None, 0)
    T = a.tokens
    out = {}
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        c = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * N * K
        r = {}
        ref = x[:2048].float() @ w.float().t()
        arms = {"hipblaslt": lambda: torch.nn.functional.linear(x, w)}
        if ext().gemm_nt_ok(x, w):
            ext().gemm_nt(x, w, c)
            r["err"] = ((c[:2048].float() - ref).abs().max() / ref.abs().max()).item()
            arms["ours"] = lambda: ext().gemm_nt(x, w, c)
        ts = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                ts[k].append(fl / timeit(fn, a.iters) / 1e12)
        for k in arms:
            r[k] = med(ts[k])
        out[name] = r
        print(name, {k: round(v, 4 if "err" in k else 1) for k, v in r.items()}, flush=True)
        del x, w, c

    # fused SwiGLU forward (gate/up GEMM + SwiGLU) and backward (down-projection dgrad + SwiGLU backward)
    F, H = 11008, 4096
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    wgu = torch.randn(2 * F, H, device="cuda", dtype=torch.bfloat16) * 0.02
    z = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    h = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    ext().gemm_nt_swiglu(x, wgu, z, h)
    ext().gemm_nt(x, wgu, zr := torch.empty_like(z))
    hr = ext().swiglu_fwd(zr[:, :F], zr[:, F:])
    zref = (x[:1024].float() @ wgu.float().t())
    hs = (torch.nn.functional.silu(zref[:, :F]) * zref[:, F:])
    fused = {"z_err": ((z[:1024].float() - zref).abs().max() / zref.abs().max()).item(),
             "h_err": ((h[:1024].float() - hs).abs().max() / hs.abs().max()).item(),
             "z_eq_unfused": bool(torch.equal(z, zr)), "h_eq_unfused": bool(torch.equal(h, hr))}
    from scaling_amd.ops import swiglu as swo
    unf = lambda: swo.swiglu_fused(torch.nn.functional.linear(x, wgu))  # noqa: E731
    fus = lambda: ext().gemm_nt_swiglu(x, wgu, z, h)  # noqa: E731
    dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    wdown = torch.randn(H, F, device="cuda", dtype=torch.bfloat16) * 0.02
    wdt = wdown.t().contiguous()
    dz = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    ext().gemm_nt_swiglu_bwd(dy, wdt, z, dz)
    dh = dy[:1024].float() @ wdown.float()
    g, u = z[:1024, :F].float().requires_grad_(), z[:1024, F:].float().requires_grad_()
    (torch.nn.functional.silu(g) * u).backward(dh)
    fused["dg_err"] = ((dz[:1024, :F].float() - g.grad).abs().max() / g.grad.abs().max()).item()
    fused["du_err"] = ((dz[:1024, F:].float() - u.grad).abs().max() / u.grad.abs().max()).item()
    dh64 = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    ext().gemm_nt(dy, wdt, dh64)
    (dz_unf,) = ext().swiglu_bwd(dh64, z[:, :F], z[:, F:], True)
    fused["dz_eq_unfused"] = bool(torch.equal(dz, dz_unf))

    def unf_bwd():
        dhh = torch.matmul(dy, wdt.t())
        return ext().swiglu_bwd(dhh, z[:, :F], z[:, F:], True)
    fus_bwd = lambda: ext().gemm_nt_swiglu_bwd(dy, wdt, z, dz)  # noqa: E731
    ts = {"swiglu_fwd_unfused": [], "swiglu_fwd_fused": [], "swiglu_bwd_unfused": [], "swiglu_bwd_fused": []}
    for _ in range(a.rounds):
        ts["swiglu_fwd_unfused"].append(timeit(unf, a.iters) * 1e3)
        ts["swiglu_fwd_fused"].append(timeit(fus, a.iters) * 1e3)
        ts["swiglu_bwd_unfused"].append(timeit(unf_bwd, a.iters) * 1e3)
        ts["swiglu_bwd_fused"].append(timeit(fus_bwd, a.iters) * 1e3)
    for k, v in ts.items():
        fused[k + "_ms"] = med(v)
    print("swiglu", {k: round(v, 4) for k, v in fused.items()}, flush=True)
    out["swiglu"] = fused
    print(json.dumps(out))


if __name__ == "__main__":
    main()
