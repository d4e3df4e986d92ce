"""GEMM probe at the 7B layer shapes as the model issues them (F.linear NT fwd, NN dgrad, TN wgrad,
weights as views into one flat buffer, addmm_ accumulation into a bf16 grad view), default hipBLASLt
heuristics vs TunableOp-tuned solutions."""
import json
import os
import sys
import time

import torch

dev = "cuda"
M = int(os.environ.get("PROBE_M", "8192"))
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "mlp_in": (22016, 4096), "mlp_out": (4096, 11008), "head": (32000, 4096)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def run(tag):
    res = {}
    flat = torch.randn(200_000_000, device=dev, dtype=torch.bfloat16)
    gflat = torch.zeros(200_000_000, device=dev, dtype=torch.bfloat16)
    off = 4096 * 3 + 64  # a realistic unaligned-to-page offset inside the flat buffer
    for name, (N, K) in SHAPES.items():
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        wv = flat[off : off + N * K].view(N, K)
        gv = gflat[off : off + N * K].view(N, K)
        g = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2 * M * N * K
        res[name] = {
            "fwd": fl / timeit(lambda: torch.nn.functional.linear(x, w)) / 1e12,
            "fwd_view": fl / timeit(lambda: torch.nn.functional.linear(x, wv)) / 1e12,
            "dgrad": fl / timeit(lambda: torch.matmul(g, w)) / 1e12,
            "wgrad": fl / timeit(lambda: torch.matmul(g.t(), x)) / 1e12,
            "wgrad_addmm_view": fl / timeit(lambda: gv.addmm_(g.t(), x)) / 1e12,
        }
        print(tag, name, {k: round(v, 1) for k, v in res[name].items()}, flush=True)
    return res


out = {"M": M, "default": run("default")}
if len(sys.argv) > 1 and sys.argv[1] == "tunable":
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(os.environ.get("TUNABLE_FILE", "gpurun_out/tunableop_results%d.csv"))
    torch.cuda.tunable.set_max_tuning_duration(200)
    out["tuned"] = run("tuned")
    torch.cuda.tunable.write_file()
print(json.dumps(out))
