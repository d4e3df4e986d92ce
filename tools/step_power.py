"""Board power / clock over the headline training step: samples ``torch.cuda.power_draw`` / ``clock_rate`` every
~10 ms on a side thread while ``bench.py`` runs (same arguments), then prints their distribution over the run.

    python tools/step_power.py --steps 5 --warmup 2
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _sample(path: str, stop) -> None:  # child process: amdsmi queries only, no HIP context
    import torch as _t

    with open(path, "w") as f:
        while not stop.is_set():
            try:
                f.write(f"{time.time()} {_t.cuda.power_draw()} {_t.cuda.clock_rate()}\n")
            except Exception:  # noqa: BLE001 - amdsmi unavailable: nothing to report
                return
            time.sleep(0.01)


def main() -> None:
    import multiprocessing as mp

    path = os.path.join(ROOT, "gpurun_out", "step_power_samples.txt")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    ctx = mp.get_context("spawn")
    stop = ctx.Event()
    child = ctx.Process(target=_sample, args=(path, stop), daemon=True)
    child.start()
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 5
    import bench

    try:
        bench.main()
    finally:
        t_ret = time.time()
        stop.set()
        child.join(timeout=5)
    # the timed steps (~1 s each at the headline shape) end just before bench.main returns (checksums + print after)
    lo, hi = t_ret - 0.5 - 0.9 * steps, t_ret - 0.5
    rows = [tuple(float(x) for x in line.split()) for line in open(path) if len(line.split()) == 3]
    tail = [r for r in rows if lo <= r[0] <= hi]
    if not tail:
        print(json.dumps({"samples": 0}))
        return
    pw = sorted(int(r[1]) for r in tail)
    ck = sorted(int(r[2]) for r in tail)

    def q(v: list[int], f: float) -> int:
        return v[min(len(v) - 1, int(f * len(v)))]

    print(json.dumps({"samples": len(tail), "window_s": round(hi - lo, 1),
                      "power_w": {"p10": q(pw, .1), "p50": q(pw, .5), "p90": q(pw, .9), "max": pw[-1]},
                      "clock_mhz": {"p10": q(ck, .1), "p50": q(ck, .5), "p90": q(ck, .9), "max": ck[-1]},
                      "frac_power_ge_1250w": round(sum(p >= 1250 for p in pw) / len(pw), 3)}))


if __name__ == "__main__":
    main()
