"""Device idle gaps of a training step from a rocprofv3 ``--hip-trace --kernel-trace --output-format csv`` run, and
what the host was doing in them.

    python tools/gap_summary.py DIR [min_gap_us]

The last complete step (between the last two AdamW clusters) is cut into kernel-busy intervals (union over all
streams); every idle interval longer than ``min_gap_us`` (default 50) is listed with the HIP API calls that were in
flight on the host during it (name histogram, longest call), so a host-side stall (synchronisation, allocation,
Python between launches) can be told apart from a device dependency."""
from __future__ import annotations

import csv
import sys
from collections import Counter
from pathlib import Path


def main() -> None:
    d = Path(sys.argv[1])
    min_gap = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 50e3  # ns
    api = next(d.rglob("*hip_api_trace.csv"))
    ker = next(d.rglob("*kernel_trace.csv"))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(ker)))
    adam = [s for s, _, n in ks if "adamw" in n]
    starts, last = [], None
    for t in adam:
        if last is None or t - last > 50_000_000:
            starts.append(t)
        last = t
    if len(starts) < 2:
        print("fewer than two optimizer steps in the trace")
        return
    t0, t1 = starts[-2], starts[-1]
    busy: list[list[int]] = []
    for s, e, _ in ks:
        if e < t0 or s > t1:
            continue
        if busy and s <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], e)
        else:
            busy.append([s, e])
    gaps = [(busy[i][1], busy[i + 1][0]) for i in range(len(busy) - 1) if busy[i + 1][0] - busy[i][1] > min_gap]
    calls = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in csv.DictReader(open(api))]
    span = (t1 - t0) / 1e6
    busy_ms = sum(e - s for s, e in busy) / 1e6
    print(f"step span {span:.1f} ms, device busy (union) {busy_ms:.1f} ms, idle {span - busy_ms:.1f} ms; "
          f"{len(gaps)} gaps > {min_gap / 1e3:.0f} us totalling {sum(b - a for a, b in gaps) / 1e6:.1f} ms")
    for a, b in sorted(gaps, key=lambda g: g[0] - g[1])[:15]:
        inside = [(s, e, f) for s, e, f in calls if e > a and s < b]
        hist = Counter(f for _, _, f in inside)
        longest = max(inside, key=lambda c: min(c[1], b) - max(c[0], a)) if inside else None
        lg = f"{longest[2]} {(longest[1] - longest[0]) / 1e3:.0f} us" if longest else "-"
        print(f"  gap {(b - a) / 1e3:8.0f} us at +{(a - t0) / 1e6:7.1f} ms: longest {lg}; calls {dict(hist.most_common(5))}")


if __name__ == "__main__":
    main()
