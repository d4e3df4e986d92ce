"""Board power / clock over the headline training step: samples ``torch.cuda.power_draw`` / ``clock_rate`` every
~10 ms on a side thread while ``bench.py`` runs (same arguments), then prints their distribution over the run.

    python tools/step_power.py --steps 5 --warmup 2
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    samples: list[tuple[float, int, int]] = []
    stop = threading.Event()

    def sampler() -> None:
        while not stop.is_set():
            try:
                samples.append((time.time(), torch.cuda.power_draw(), torch.cuda.clock_rate()))
            except Exception:  # noqa: BLE001 - amdsmi unavailable: nothing to report
                return
            time.sleep(0.01)

    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
    import bench

    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    t0 = time.time()
    try:
        bench.main()
    finally:
        stop.set()
        th.join(timeout=2)
    # the timed steps (~1 s each at the headline shape) end the run: keep the last 0.9 s per timed step
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 5
    t_end = samples[-1][0] if samples else time.time()
    tail = [s for s in samples if s[0] > max(t0, t_end - 0.9 * steps)]
    if not tail:
        print(json.dumps({"samples": 0}))
        return
    pw = sorted(s[1] for s in tail)
    ck = sorted(s[2] for s in tail)

    def q(v: list[int], f: float) -> int:
        return v[min(len(v) - 1, int(f * len(v)))]

    print(json.dumps({"samples": len(tail),
                      "power_w": {"p10": q(pw, .1), "p50": q(pw, .5), "p90": q(pw, .9), "max": pw[-1]},
                      "clock_mhz": {"p10": q(ck, .1), "p50": q(ck, .5), "p90": q(ck, .9), "max": ck[-1]},
                      "frac_power_ge_1250w": round(sum(p >= 1250 for p in pw) / len(pw), 3)}))


if __name__ == "__main__":
    main()
