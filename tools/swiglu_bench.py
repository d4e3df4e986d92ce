"""SwiGLU forward / backward kernels at the 7B MLP shape (T 32768, F 11008): GB/s and an output fingerprint (run under
two builds with SCALING_AMD_EXT_SO to A/B a kernel change; the fingerprints must agree)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

T, F = 32768, 11008
g = torch.Generator(device="cuda").manual_seed(7)
z = torch.randn(T, 2 * F, device="cuda", generator=g).to(torch.bfloat16)
dy = torch.randn(T, F, device="cuda", generator=g).to(torch.bfloat16)
a, b = z[:, :F], z[:, F:]


def timed(fn, iters=10):
    for _ in range(3):
        out = fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        out = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters, out


dig = lambda t: hashlib.sha1(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]
for _ in range(3):
    ms_f, h = timed(lambda: ext().swiglu_fwd(a, b))
    ms_b, (dz,) = timed(lambda: ext().swiglu_bwd(dy, a, b, True))
    print(f"fwd {ms_f:.3f} ms {3 * T * F * 2 / ms_f / 1e6:.0f} GB/s | bwd {ms_b:.3f} ms {5 * T * F * 2 / ms_b / 1e6:.0f} GB/s | "
          f"h {dig(h)} dz {dig(dz)}", flush=True)
