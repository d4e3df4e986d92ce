"""Does the shipped TunableOp table (``scaling_amd/tuning/gemm_gfx950.csv``) serve the step's forward GEMMs?

Times the 7B forward / dgrad shapes the way the training step issues them (``F.linear`` on the 3-D activation, and
``a @ (W^T)^T`` for the dgrad through the cached transpose), with TunableOp on (table loaded, tuning off) and off
(library heuristic), and prints how many table rows TunableOp holds after the calls.

    PYTORCH_TUNABLEOP_VERBOSE=1 python tools/gemm_table_check.py
"""
from __future__ import annotations

import json
import statistics

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from scaling_amd.utils.gemm_tuning import enable_tuned_gemms

SHAPES = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}


def _time(fn, iters: int = 12) -> float:
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main() -> None:
    mode = enable_tuned_gemms("use", None, 0)
    tun = torch.cuda.tunable
    print(json.dumps({"mode": mode, "filename": tun.get_filename(), "validators": [list(v) for v in tun.get_validators()]}))
    B, S = 8, 4096
    res = {}
    for name, (k, n) in SHAPES.items():
        x3 = torch.randn(B, S, k, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = w.t().contiguous()
        g = torch.randn(B * S, n, device="cuda", dtype=torch.bfloat16)
        row = {}
        for on in (True, False):
            tun.enable(on)
            tag = "table" if on else "heuristic"
            row[f"fwd3d_{tag}"] = _time(lambda: torch.nn.functional.linear(x3, w))
            row[f"fwd2d_{tag}"] = _time(lambda: torch.nn.functional.linear(x3.view(-1, k), w))
            row[f"dgrad_{tag}"] = _time(lambda: torch.matmul(g, wt.t()))
        tun.enable(True)
        res[name] = {kk: round(v, 4) for kk, v in row.items()}
        print(name, json.dumps(res[name]), flush=True)
        del x3, w, wt, g
    results = tun.get_results()
    print(json.dumps({"table_rows_loaded": len(results),
                      "rows_32768": [list(r) for r in results if "32768" in str(r[1])]}))


if __name__ == "__main__":
    main()
