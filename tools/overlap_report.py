"""Which kernels / memory copies of the same process run at the same time as a given kernel (race forensics).

    python tools/overlap_report.py <rocprofv3 csv output dir> [kernel-name substring, default fa_bwd]

Reads every ``*kernel_trace.csv`` (and ``*memory_copy_trace.csv``) under the directory (rocprofv3 --kernel-trace
--memory-copy-trace --output-format csv, one set per process), and for each dispatch whose name contains the substring
lists the other dispatches / copies of the SAME process whose [start, end) intersects it, grouped by name and
queue/stream.
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import Counter, defaultdict


def _rows(pattern: str) -> list[dict]:
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def _key(r: dict, *names: str) -> str:
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    return "?"


def main() -> None:
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "fa_bwd"
    ks = _rows(os.path.join(d, "**", "*kernel_trace.csv"))
    cs = _rows(os.path.join(d, "**", "*memory_copy_trace.csv"))
    ev = []
    for r in ks:
        ev.append(("kernel", _key(r, "Process_Id", "Pid"), _key(r, "Stream_Id", "Queue_Id"), _key(r, "Kernel_Name"),
                   int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for r in cs:
        ev.append(("copy", _key(r, "Process_Id", "Pid"), _key(r, "Stream_Id", "Queue_Id"),
                   _key(r, "Direction", "Operation", "Kind"), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    by_pid = defaultdict(list)
    for e in ev:
        by_pid[e[1]].append(e)
    for pid, es in sorted(by_pid.items()):
        es.sort(key=lambda e: e[4])
        targets = [e for e in es if e[0] == "kernel" and sub in e[3]]
        over = Counter()
        hits = 0
        for t in targets:
            found = False
            for e in es:
                if e is t or e[4] >= t[5] or e[5] <= t[4]:
                    continue
                if e[0] == "kernel" and e[2] == t[2]:
                    continue  # same stream: ordered
                over[(e[0], e[2], e[3][:80])] += 1
                found = True
            hits += found
        print(f"process {pid}: {len(targets)} '{sub}' dispatches, {hits} overlapped by another stream's work")
        for (kind, q, name), n in over.most_common(15):
            print(f"   {n:5d}  {kind:6s} stream/queue {q}: {name}")


if __name__ == "__main__":
    main()
