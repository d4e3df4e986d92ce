"""Synchronizing HIP API calls per training step from a rocprofv3 ``--hip-trace --kernel-trace`` CSV run.

    python tools/sync_trace_summary.py DIR

Step boundaries are the AdamW launches (the last kernels of an optimizer step).  For every step interval it
counts device-wide waits (hipDeviceSynchronize), host waits on a stream or event and blocking copies."""
from __future__ import annotations

import csv
import sys
from collections import Counter
from pathlib import Path

SYNC = ("hipDeviceSynchronize", "hipStreamSynchronize", "hipEventSynchronize", "hipMemcpy", "hipMemcpyWithStream",
        "hipStreamQuery", "hipEventQuery")


def main() -> None:
    d = Path(sys.argv[1])
    api = next(d.rglob("*hip_api_trace.csv"))
    ker = next(d.rglob("*kernel_trace.csv"))
    adam = sorted(int(r["Start_Timestamp"]) for r in csv.DictReader(open(ker)) if "adamw" in r["Kernel_Name"])
    # optimizer steps: clusters of AdamW launches
    steps, last = [], None
    for t in adam:
        if last is None or t - last > 50_000_000:  # > 50 ms apart: a new step
            steps.append(t)
        last = t
    calls = [(int(r["Start_Timestamp"]), r["Function"]) for r in csv.DictReader(open(api)) if r["Function"].startswith(SYNC)]
    print(f"optimizer steps found: {len(steps)} (AdamW clusters)")
    for i in range(len(steps) - 1):
        c = Counter(f for t, f in calls if steps[i] <= t < steps[i + 1])
        print(f"step {i + 1} -> {i + 2}: " + (", ".join(f"{k} x{v}" for k, v in sorted(c.items())) or "no synchronizing call"))
    tot = Counter(f for _, f in calls)
    print("whole run: " + ", ".join(f"{k} x{v}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
