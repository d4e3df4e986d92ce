"""Per-kernel PMC summary from rocprofv3 ``--output-format csv`` counter files.

    python tools/pmc_csv_summary.py DIR_OR_CSV [DIR_OR_CSV ...] [--match SUBSTR]

Counters are averaged per dispatch and kernel (name truncated at the argument list).  Derived rows:
  * VALU/MFMA, LDS/MFMA (instruction ratios) when SQ_INSTS_* are present;
  * MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
    (MFMA busy cycles are summed over all SIMDs; GUI_ACTIVE is summed over the 8 XCDs);
  * clock = GRBM_GUI_ACTIVE / 8 / kernel wall time (MHz, DVFS check);
  * wait fractions of SQ_WAVE_CYCLES.
"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def _files(args: list[str]) -> list[Path]:
    out = []
    for a in args:
        p = Path(a)
        out.extend(sorted(p.rglob("*counter_collection.csv")) if p.is_dir() else [p])
    return out


def main() -> None:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = ""
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args.remove(match)
    vals: dict[str, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
    wall: dict[str, dict[int, float]] = defaultdict(dict)
    for f in _files(args):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:70]
                if match not in name:
                    continue
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                wall[name][int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    order = sorted(vals, key=lambda k: -sum(wall[k].values()))  # heaviest kernels first
    for name in order:
        cs = vals[name]
        n = len(wall[name])
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        t = sum(wall[name].values()) / max(1, n)
        print(f"{name}  dispatches {n}  mean {t * 1e3:.3f} ms")
        print("   ", {c: round(v) for c, v in sorted(avg.items())})
        d = []
        if avg.get("SQ_INSTS_MFMA"):
            if "SQ_INSTS_VALU" in avg:
                d.append(f"VALU/MFMA {avg['SQ_INSTS_VALU'] / avg['SQ_INSTS_MFMA']:.2f}")
            if "SQ_INSTS_LDS" in avg:
                d.append(f"LDS/MFMA {avg['SQ_INSTS_LDS'] / avg['SQ_INSTS_MFMA']:.2f}")
        if avg.get("SQ_VALU_MFMA_BUSY_CYCLES") and avg.get("GRBM_GUI_ACTIVE"):
            d.append(f"MFMA util {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
        if avg.get("GRBM_GUI_ACTIVE") and t > 0:
            d.append(f"clock {avg['GRBM_GUI_ACTIVE'] / 8 / t / 1e6:.0f} MHz")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if k in avg:
                    d.append(f"{k[3:]}/WAVE {avg[k] / wc:.3f}")
        if avg.get("FETCH_SIZE") and t > 0:  # FETCH_SIZE is in KiB
            d.append(f"HBM read {avg['FETCH_SIZE'] * 1024 / t / 1e12:.2f} TB/s")
        if avg.get("SQ_LDS_BANK_CONFLICT") is not None and avg.get("SQ_LDS_IDX_ACTIVE"):
            d.append(f"LDS conflict/active {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f}")
        if d:
            print("    " + "  ".join(d))


if __name__ == "__main__":
    main()
