"""Summarise a rocprofv3 rocpd database (kernel trace) into a per-kernel table (markdown).

usage: python tools/rocpd_summary.py <run_results.db> [--top N] [--steps K]
Kernel names are shortened; hipBLASLt/Tensile GEMMs are grouped by macro tile.
"""
from __future__ import annotations

import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        m = re.search(r"(Cijk_A\w{3}_B\w{3}).*?(MT\d+x\d+x\d+)", name)
        return f"GEMM {m.group(1)} {m.group(2)}" if m else "GEMM"
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--steps", type=int, default=1, help="divide totals by this many profiled steps")
    ap.add_argument("--tail-ms", type=float, default=None,
                    help="only kernels that start within the last this-many ms of the trace (e.g. a graph replay phase)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end from kernels"))
    if a.tail_ms is not None:
        end = max(r[2] for r in rows)
        rows = [r for r in rows if r[1] >= end - a.tail_ms * 1e6]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    for n, s, e in rows:
        k = short(n)
        tot[k] += (e - s) / 1e6
        cnt[k] += 1
    busy = sum(tot.values())
    print(f"kernels: {len(rows)}  busy {busy:.1f} ms  span {(t1 - t0) / 1e6:.1f} ms  (per step /{a.steps})\n")
    print("| kernel | calls | total ms | avg us | % busy |")
    print("|---|---|---|---|---|")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[: a.top]:
        print(f"| {k} | {cnt[k] / a.steps:.0f} | {v / a.steps:.2f} | {1000 * v / cnt[k]:.1f} | {100 * v / busy:.1f} |")


if __name__ == "__main__":
    main()
