"""Does ``torch.bmm`` run the strided token pieces of ``tp_overlap.py`` as ONE vendor GEMM without copies?

A sequence-parallel piece is ``size`` blocks of R rows with a block stride of ``chunks * R`` rows (a ``[size, R, K]``
view with batch stride ``chunks*R*K``); the weight is shared (batch stride 0 via ``expand``).  For each variant the
script times the product and lists the kernels the profiler saw (a copy / elementwise kernel next to the GEMM means
torch materialised an operand).

    python tools/bmm_stride_probe.py
"""
from __future__ import annotations

import json

import torch


def main() -> None:
    dev = torch.device("cuda")
    size, chunks, R, K, N = 2, 4, 2048, 4096, 4096
    T = size * chunks * R
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    x4 = x.view(size, chunks, R, K)
    out = torch.empty(size, chunks, R, N, device=dev, dtype=torch.bfloat16)
    wT = w.t()
    i = 1

    variants = {
        "mm contiguous [size*R,K] (reference speed)": lambda: torch.mm(x[: size * R], wT),
        "matmul strided piece (current fwd)": lambda: torch.matmul(x4[:, i], wT),
        "bmm strided piece, expanded W": lambda: torch.bmm(x4[:, i], wT.unsqueeze(0).expand(size, K, N)),
        "bmm strided piece -> strided out": lambda: torch.bmm(x4[:, i], wT.unsqueeze(0).expand(size, K, N),
                                                            out=out[:, i]),
        "per-rank mm x size (current bwd)": lambda: [torch.mm(x4[r, i], wT, out=out[r, i]) for r in range(size)],
    }
    ref = torch.matmul(x4[:, i].float(), wT.float())
    for name, fn in variants.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            fn()
            torch.cuda.synchronize()
        kernels = sorted({e.name[:90] for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA})
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        res = fn()
        if isinstance(res, list):
            res = out[:, i]
        err = None
        if "reference" not in name:
            err = round((res.float() - ref).abs().max().item() / ref.abs().max().item(), 5)
        print(json.dumps({"variant": name, "us": round(s.elapsed_time(e) / 20 * 1000, 1),
                          "tflops": round(2 * size * R * K * N / (s.elapsed_time(e) / 20 / 1000) / 1e12, 1),
                          "rel_err": err, "kernels": kernels}), flush=True)


if __name__ == "__main__":
    main()
