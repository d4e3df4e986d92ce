"""Attention-only driver for kernel profiling (7B step shapes): B=8 (env B), S=4096, Hq=32, Hkv=8, D=128, causal
(CAUSAL=0: full attention)."""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops import attention  # noqa: E402

B, S, HQ, HK, D = int(os.environ.get("B", 8)), 4096, int(os.environ.get("HQ", 32)), int(os.environ.get("HKV", 8)), 128
iters = int(os.environ.get("ITERS", 5))
CAUSAL = os.environ.get("CAUSAL", "1") != "0"
T = B * S
cu = torch.arange(0, T + 1, S, device="cuda", dtype=torch.int32)
if os.environ.get("PACKED") == "1":  # q / k / v as views of one [T, Hq + 2 Hkv, D] projection output, as in training
    base = torch.randn(T, HQ + 2 * HK, D, device="cuda", dtype=torch.bfloat16)
    q = base[:, :HQ].detach().requires_grad_(True)
    k = base[:, HQ:HQ + HK].detach().requires_grad_(True)
    v = base[:, HQ + HK:].detach().requires_grad_(True)
else:
    q = torch.randn(T, HQ, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(T, HK, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(T, HK, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
g = torch.randn(T, HQ, D, device="cuda", dtype=torch.bfloat16)
sc = 1 / math.sqrt(D)

def once():
    for _ in range(2):
        o = attention.flash_attention(q, k, v, cu, cu, S, S, sc, CAUSAL, None)
        o.backward(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        o = attention.flash_attention(q, k, v, cu, cu, S, S, sc, CAUSAL, None)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(iters):
        o = attention.flash_attention(q, k, v, cu, cu, S, S, sc, CAUSAL, None)
        o.backward(g)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    fwd = (t1 - t0) / iters
    tot = (t2 - t1) / iters
    fl = 4 * B * HQ * S * S * D / (2 if CAUSAL else 1)
    return f"fwd {fwd*1e3:.3f} ms {fl/fwd/1e12:.0f} TF | bwd {(tot-fwd)*1e3:.3f} ms {2.5*fl/(tot-fwd)/1e12:.0f} TF(2.5x)"


for _ in range(3):
    print(once(), flush=True)
