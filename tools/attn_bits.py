"""Bit fingerprint of the flash-attention kernels (forward output + LSE, backward dQ / dK / dV) over fixed-seed inputs of
several layouts (causal / full, sliding window, GQA, varlen, D 64 / 128): run it under two builds
(``SCALING_AMD_EXT_SO``) and diff the printed lines to check that a kernel change is bit-identical.

usage: python tools/attn_bits.py
"""
import hashlib
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops import attention  # noqa: E402


def digest(t: torch.Tensor) -> str:
    return hashlib.sha1(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]


CASES = [  # (segment lengths, Hq, Hkv, D, causal, window)
    ([4096, 4096], 32, 8, 128, True, None),
    ([1000, 3000, 777], 8, 2, 128, True, None),
    ([2048], 8, 8, 128, False, None),
    ([3000, 1100], 8, 4, 128, True, 500),
    ([1500], 4, 1, 64, True, None),
    ([2000, 300], 4, 2, 64, False, 256),
]

for lens, hq, hk, d, causal, window in CASES:
    g = torch.Generator(device="cuda").manual_seed(1234 + len(lens) * 7 + hq + d)
    T = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0).tolist()), device="cuda", dtype=torch.int32)
    mk = lambda h: (torch.randn(T, h, d, device="cuda", generator=g) * 1.5).to(torch.bfloat16).requires_grad_(True)
    q, k, v = mk(hq), mk(hk), mk(hk)
    do = torch.randn(T, hq, d, device="cuda", generator=g).to(torch.bfloat16)
    o = attention.flash_attention(q, k, v, cu, cu, max(lens), max(lens), 1 / math.sqrt(d), causal, window)
    o.backward(do)
    torch.cuda.synchronize()
    print(f"lens={lens} hq={hq} hk={hk} d={d} causal={causal} window={window}: o {digest(o)} dq {digest(q.grad)} "
          f"dk {digest(k.grad)} dv {digest(v.grad)}", flush=True)
