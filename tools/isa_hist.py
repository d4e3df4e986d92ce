"""Per-basic-block instruction histogram of a gfx950 kernel (hipcc -S of one .hip file).

Usage: python tools/isa_hist.py csrc/kernels/flash_fwd.hip fa_fwd_v2_kernel [--all-blocks] [--flags "-DX=1"]

Compiles the file for the device only (same flags as the extension build), picks the kernels whose (mangled or
demangled) name contains the filter, splits each into basic blocks at its labels and prints, for every block that
issues MFMAs (or every block with --all-blocks), the count per class:
  mfma, valu (non-MFMA vector ALU), trans (v_exp/v_log/v_rcp/v_rsq/v_sqrt/v_sin/v_cos), pk (v_pk_*), cvt,
  perm (v_permlane*, ds_bpermute/swizzle), ds_rd, ds_wr, vmem (buffer/global loads+stores, LDS-DMA), salu, wait
  (s_waitcnt), nop (s_nop), barrier, branch.
and the non-MFMA VALU per MFMA ratio of the block.  The loop body of an attention kernel is the block (or the blocks)
with the most MFMAs; --all-blocks shows the prologue/epilogue too.
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def classify(op: str) -> str:
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_pk_"):
        return "pk"
    if op.startswith("v_cvt"):
        return "cvt"
    if op.startswith("v_permlane") or op in ("ds_bpermute_b32", "ds_permute_b32") or op.startswith("ds_swizzle"):
        return "perm"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_rd"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "ds_wr"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op == "s_nop":
        return "nop"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


COLS = ["mfma", "valu", "trans", "pk", "cvt", "perm", "accmov", "ds_rd", "ds_wr", "vmem", "salu", "wait", "nop",
        "barrier", "branch"]


def compile_asm(src: str, defs: list[str]) -> str:
    out = "/tmp/isa_hist.s"
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-S",
           "-x", "hip", f"-I{ROOT}/csrc", f"-I{ROOT}/csrc/kernels", "-D__HIP_PLATFORM_AMD__=1", *defs, src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(r.stderr)
    return open(out).read()


def kernels(asm: str) -> dict[str, list[str]]:
    res: dict[str, list[str]] = {}
    cur = None
    for line in asm.splitlines():
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith((".L", "$")):
            cur = m.group(1)
            res[cur] = []
            continue
        if cur is not None:
            if line.startswith("\t.end_amdhsa_kernel") or re.match(r"^\.Lfunc_end", line):
                cur = None
                continue
            res[cur].append(line)
    return res


def blocks(lines: list[str]) -> list[tuple[str, collections.Counter]]:
    out = []
    name, cnt = "entry", collections.Counter()
    for line in lines:
        m = re.match(r"^(\.L\w+):", line) or re.match(r"^; (%bb\.\d+):", line)
        if m:
            out.append((name, cnt))
            name, cnt = m.group(1), collections.Counter()
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        cnt[classify(op)] += 1
    out.append((name, cnt))
    return out


def demangle(n: str) -> str:
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("filter")
    ap.add_argument("--all-blocks", action="store_true")
    ap.add_argument("--flags", default="", help="extra compiler flags, one string (e.g. \"-DX=1 -mllvm -opt\")")
    a = ap.parse_args()
    asm = compile_asm(a.src, a.flags.split())
    for k, lines in kernels(asm).items():
        dn = demangle(k)
        if a.filter not in k and a.filter not in dn:
            continue
        print(f"== {dn}")
        print(f"{'block':>12s} " + " ".join(f"{c:>7s}" for c in COLS) + "  valu/mfma (valu+trans+pk+cvt+perm)")
        tot = collections.Counter()
        for name, c in blocks(lines):
            tot += c
            if not a.all_blocks and c["mfma"] == 0:
                continue
            nm = sum(c[x] for x in ("valu", "trans", "pk", "cvt", "perm"))
            ratio = f"{nm / c['mfma']:.2f}" if c["mfma"] else "-"
            print(f"{name:>12s} " + " ".join(f"{c[x]:7d}" for x in COLS) + f"  {ratio}")
        nm = sum(tot[x] for x in ("valu", "trans", "pk", "cvt", "perm"))
        print(f"{'total':>12s} " + " ".join(f"{tot[x]:7d}" for x in COLS) +
              (f"  {nm / tot['mfma']:.2f}" if tot["mfma"] else ""))


if __name__ == "__main__":
    main()
