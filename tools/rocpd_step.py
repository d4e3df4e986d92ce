"""Per-step kernel time breakdown from a rocprofv3 rocpd database: steps are delimited by the optimizer's
fused AdamW launches; reports the last complete step's kernels grouped by category (ms) and the GPU-busy
vs wall span of that step.

usage: python tools/rocpd_step.py <run_results.db>
"""
from __future__ import annotations

import bisect
import re
import sqlite3
import sys
from collections import defaultdict


def category(name: str) -> str:
    rules = [("Cijk", "hipBLASLt GEMM"), ("gemm_tn", "wgrad GEMM (HIP)"), ("fa_fwd", "attention fwd"),
             ("fa_bwd_dkdv", "attention bwd dK/dV"), ("fa_bwd_dq", "attention bwd dQ"), ("fa_bwd", "attention bwd other"),
             ("adamw", "AdamW"), ("swiglu", "SwiGLU"), ("norm_", "norm"), ("colsum", "norm"), ("rope", "RoPE"),
             ("xent", "cross-entropy"), ("embed", "embedding"), ("transpose_u16", "W^T transpose"),
             ("sumsq", "grad norm"), ("cast_scale", "grad cast"), ("rccl", "RCCL"), ("nccl", "RCCL")]
    for key, cat in rules:
        if key in name:
            return cat
    return "other: " + re.sub(r"\(.*", "", name)[:60]


def main() -> None:
    c = sqlite3.connect(sys.argv[1])
    rows = sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])
    adam = [i for i, r in enumerate(rows) if "adamw" in r[0]]
    # step boundary = first kernel after a run of AdamW launches
    ends = [i for j, i in enumerate(adam) if j + 1 == len(adam) or adam[j + 1] - i > 50]
    if len(ends) < 2:
        print("need two complete steps in the trace")
        return
    # the last window whose AdamW run is followed by another step's forward (the overlapped update runs beside it)
    lo, hi = (ends[-3] + 1, ends[-2] + 1) if len(ends) > 2 else (ends[-2] + 1, ends[-1] + 1)
    step = rows[lo:hi]
    tot = defaultdict(float)
    for name, s, e in step:
        tot[category(name)] += (e - s) / 1e6
    busy = sum(tot.values())
    span = (max(e for _, _, e in step) - step[0][1]) / 1e6
    union, cur = 0, None  # device-busy time: union of kernel intervals over all streams
    for _, s, e in step:
        if cur is None or s > cur[1]:
            if cur is not None:
                union += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur is not None:
        union += cur[1] - cur[0]
    # NB the window runs from the first kernel after one AdamW run to the last AdamW launch of the next: with the
    # overlapped optimizer step those launches interleave with the next forward, so span - union can include
    # device time outside the window; tools/gap_summary.py measures idle time from a HIP API + kernel trace
    print(f"last complete step: {len(step)} kernels, kernel time {busy:.1f} ms, device busy (union) "
          f"{union / 1e6:.1f} ms, span {span:.1f} ms")
    # how much of the optimizer update ran beside other kernels (the overlapped step's point): AdamW time covered by
    # the union of every non-AdamW kernel interval of the whole trace
    others, cur = [], None
    for name, s, e in rows:
        if "adamw" in name:
            continue
        if cur is None or s > cur[1]:
            if cur is not None:
                others.append(cur)
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur is not None:
        others.append(cur)
    adam_win = [(s, e) for name, s, e in step if "adamw" in name]
    starts = [o[0] for o in others]
    cov = 0
    for s, e in adam_win:
        i = max(bisect.bisect_right(starts, s) - 1, 0)
        while i < len(others) and others[i][0] < e:
            cov += max(0, min(e, others[i][1]) - max(s, others[i][0]))
            i += 1
    adam_t = sum(e - s for s, e in adam_win)
    if adam_win:
        print(f"AdamW of the step: {adam_t / 1e6:.1f} ms kernel time, {cov / 1e6:.1f} ms of it beside other kernels; "
              f"first AdamW {(adam_win[0][0] - step[0][1]) / 1e6:.1f} ms after the window start")
    print("| category | ms | % of busy |\n|---|---|---|")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"| {k} | {v:.1f} | {100 * v / busy:.1f} |")
    if len(sys.argv) > 2:  # top-N kernels of the step by full name
        per: dict[str, list[float]] = defaultdict(lambda: [0, 0.0])
        for name, s, e in step:
            per[name][0] += 1
            per[name][1] += (e - s) / 1e6
        print(f"\n| kernel (top {sys.argv[2]}) | calls | ms |\n|---|---|---|")
        for k, (n, v) in sorted(per.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[2])]:
            print(f"| {k[:150]} | {n} | {v:.1f} |")


if __name__ == "__main__":
    main()
