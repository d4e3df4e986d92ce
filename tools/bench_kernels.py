"""Micro-benchmarks of the HIP kernels at Llama-2-7B shapes (one process, interleaved rounds)."""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops import attention, norm, rope, swiglu, xent  # noqa: E402

dev = "cuda"
res = {}


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


B, S, H, HK, D = 4, 4096, 32, int(os.environ.get("HKV", 32)), 128
T = B * S
q = torch.randn(T, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(T, HK, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(T, HK, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
cu = torch.arange(0, T + 1, S, device=dev, dtype=torch.int32)
flops_fwd = 4 * B * H * S * S * D / 2  # causal
dt = timeit(lambda: attention.flash_attention(q, k, v, cu, cu, S, S, None, True))
res["attn_fwd_causal_TF"] = flops_fwd / dt / 1e12
o = attention.flash_attention(q, k, v, cu, cu, S, S, None, True)
g = torch.randn_like(o)
dt2 = timeit(lambda: torch.autograd.grad(o, (q, k, v), g, retain_graph=True), iters=5)
res["attn_bwd_causal_TF(2.5x fwd flops)"] = 2.5 * flops_fwd / dt2 / 1e12
res["attn_fwd_ms"] = dt * 1e3
res["attn_bwd_ms"] = dt2 * 1e3
print(res, flush=True)

x = torch.randn(T, 4096, device=dev, dtype=torch.bfloat16, requires_grad=True)
w = torch.ones(4096, device=dev, dtype=torch.bfloat16, requires_grad=True)
dt = timeit(lambda: norm.rms_norm(x, w, 1e-5))
res["rmsnorm_fwd_GBs"] = 2 * x.numel() * 2 / dt / 1e9
y = norm.rms_norm(x, w, 1e-5)
gy = torch.randn_like(y)
dt = timeit(lambda: torch.autograd.grad(y, (x, w), gy, retain_graph=True))
res["rmsnorm_bwd_GBs"] = 3 * x.numel() * 2 / dt / 1e9
z = torch.randn(T, 2 * 11008, device=dev, dtype=torch.bfloat16, requires_grad=True)
dt = timeit(lambda: swiglu.swiglu_fused(z))
res["swiglu_fwd_GBs"] = 1.5 * z.numel() * 2 / dt / 1e9
cos, sin = rope.rope_tables(128, S, 10000, True, torch.bfloat16, dev)
qkv = torch.randn(T, 3 * H, D, device=dev, dtype=torch.bfloat16)
dt = timeit(lambda: rope.apply_rope(qkv[:, :H], cos, sin, None, 128, S, True))
res["rope_GBs"] = 2 * T * H * D * 2 / dt / 1e9
logits = torch.randn(T // 2, 32000, device=dev, dtype=torch.bfloat16)
tgt = torch.randint(0, 32000, (T // 2,), device=dev)
dt = timeit(lambda: xent.vocab_parallel_cross_entropy(logits, tgt))
res["xent_fwd_GBs"] = logits.numel() * 2 / dt / 1e9
print(json.dumps(res, indent=1), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/bench_kernels.json", "w"), indent=1)
