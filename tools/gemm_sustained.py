"""Sustained-load GEMM rate: one hipBLASLt shape of the 7B step called back to back for a few seconds.

Answers whether the gap between the tuning table's per-call times (short, isolated bursts) and the same GEMMs inside
the training step is the clock the chip holds under sustained load: each call is timed with HIP events and the rate
is reported per ~100 ms window, with the SMU's clock / power where torch can read them.

    python tools/gemm_sustained.py [--shape gate_up|down|qkv|o|head] [--seconds 3]
"""
from __future__ import annotations

import argparse
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # (tokens, in, out) of F.linear(x[tokens, in], W[out, in])
    "qkv": (32768, 4096, 6144),
    "o": (32768, 4096, 4096),
    "gate_up": (32768, 4096, 22016),
    "down": (32768, 11008, 4096),
    "head": (32768, 4096, 32000),
}


def _smu() -> dict:
    out = {}
    for name in ("clock_rate", "power_draw", "temperature"):
        fn = getattr(torch.cuda, name, None)
        if fn is None:
            continue
        try:
            out[name] = fn()
        except Exception:  # noqa: BLE001 - amdsmi missing or not permitted on the box
            pass
    return out


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--shape", default="gate_up", choices=sorted(SHAPES))
    p.add_argument("--seconds", type=float, default=3.0)
    p.add_argument("--idle-first", type=float, default=2.0, help="sleep before the run so the chip starts cool")
    a = p.parse_args()
    from scaling_amd.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms("use", None, 0)
    t, k, n = SHAPES[a.shape]
    x = torch.randn(t, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
    y = torch.nn.functional.linear(x, w)  # tuning-table lookup / first-call setup
    torch.cuda.synchronize()
    time.sleep(a.idle_first)
    flop = 2.0 * t * k * n
    ev = []
    t0 = time.time()
    while time.time() - t0 < a.seconds:
        batch = []
        for _ in range(8):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            y = torch.nn.functional.linear(x, w)
            e.record()
            batch.append((s, e))
        torch.cuda.synchronize()
        smu = _smu()
        for s, e in batch:
            ev.append((time.time() - t0, s.elapsed_time(e), smu))
    first = [ms for _, ms, _ in ev[:5]]
    print(json.dumps({"shape": a.shape, "calls": len(ev), "first5_ms": [round(v, 4) for v in first],
                      "table_hint": "scaling_amd/tuning/gemm_gfx950.csv"}))
    win, acc = 0.1, []
    for wall, ms, smu in ev:
        acc.append(ms)
        if wall >= win:
            mean = sum(acc) / len(acc)
            print(json.dumps({"t_s": round(wall, 2), "calls": len(acc), "mean_ms": round(mean, 4),
                              "tflops": round(flop / mean / 1e9, 1), **smu}))
            acc, win = [], win + 0.1


if __name__ == "__main__":
    main()
