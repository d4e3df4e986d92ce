"""Static check of the LDS-DMA hand-off rules in the attention kernels (the race the round-5 gradient trace found).

* RAW: every ``s_barrier`` after which waves read tiles that OTHER waves staged by LDS-DMA must be preceded, in each
  wave, by an ``s_waitcnt vmcnt(0)`` with no LDS-DMA issue in between (``flash_attn.h: dma_barrier``).
* WAR: no LDS-DMA may be issued into LDS that a wave may still be reading: walking back from every LDS-DMA issue along
  every control-flow path (fall-through and branches into each block), an ``s_barrier`` must come before any
  ``ds_read*``, and behind that barrier an ``s_waitcnt ... lgkmcnt(0)`` before any earlier ``ds_read*`` -- so every
  wave's reads have returned before any wave overwrites (all waves run the same code).  Paths that reach the kernel
  entry (the prologue) are fine.  Slot-blind, so it is conservative: a DMA into a slot nobody reads would also have to
  be separated.
Compiles the kernel files to gfx950 assembly (the extension build's flags) and walks the listed kernels.

    python tools/dma_barrier_check.py      # exit 1 and a list of offending barriers on failure
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = {"flash_fwd.hip": ("fa_fwd_v2_kernel",), "flash_bwd.hip": ("fa_bwd_dkdv_kernel", "fa_bwd_dq_kernel")}
sys.path.insert(0, ROOT)
from scaling_amd._build import _FILE_FLAGS as FLAGS  # noqa: E402  (the extension build's per-file flags)


def check_file(name: str, kernels: tuple[str, ...]) -> list[str]:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-S", "-x",
               "hip", f"-I{ROOT}/csrc", f"-I{ROOT}/csrc/kernels", *FLAGS.get(name, []),
               os.path.join(ROOT, "csrc", "kernels", name), "-o", out]
        subprocess.run(cmd, check=True, capture_output=True)
        s = open(out).read()
    bad = []
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        fn = m.group(1)
        if not any(k in fn for k in kernels):
            continue
        body = s[m.end(): s.index(".Lfunc_end", m.end())].splitlines()
        bad += war_violations(name, fn, body)
        for n, line in enumerate(body):
            if line.strip() != "s_barrier":
                continue
            for k in range(n - 1, -1, -1):
                t = body[k].strip()
                if "vmcnt(0)" in t:
                    break
                if t.startswith(("buffer_load", "global_load_lds")) and " lds" in t:
                    bad.append(f"{name}:{fn}: barrier at line {n} has an LDS-DMA issue after the last vmcnt(0)")
                    break
    return bad


_BRANCH = re.compile(r"^s_(?:cbranch_\w+|branch)\s+(\.\w+)")


def _is_dma(t: str) -> bool:
    return t.startswith(("buffer_load", "global_load_lds")) and " lds" in t


def war_violations(name: str, fn: str, body: list[str]) -> list[str]:
    """WAR rule (module docstring) for one kernel body."""
    lines = [ln.strip() for ln in body]
    labels = {t[:-1]: i for i, t in enumerate(lines) if re.match(r"^\.\w+:$", t)}
    sites: dict[str, list[int]] = {}
    for i, t in enumerate(lines):
        m = _BRANCH.match(t)
        if m:
            sites.setdefault(m.group(1), []).append(i)

    def walk(k: int, barrier: bool, seen: set) -> bool:
        """True if every path backwards from line k (exclusive) satisfies the rule in state ``barrier``."""
        while k > 0:
            k -= 1
            t = lines[k]
            if t.endswith(":") and t[:-1] in labels:
                key = (t[:-1], barrier)
                if key in seen:
                    return True
                seen.add(key)
                if not all(walk(j, barrier, seen) for j in sites.get(t[:-1], [])):
                    return False
                prev = lines[k - 1] if k > 0 else ""
                if prev.startswith(("s_branch", "s_endpgm")):
                    return True  # no fall-through into this block
                continue
            if t.startswith("ds_read"):
                return False
            if not barrier and t == "s_barrier":
                barrier = True
            elif barrier and t.startswith("s_waitcnt") and "lgkmcnt(0)" in t:
                return True
        return True

    bad = []
    for i, t in enumerate(lines):
        if _is_dma(t) and not walk(i, False, set()):
            bad.append(f"{name}:{fn}: LDS-DMA at line {i} may overwrite LDS that a wave has not finished reading")
    return bad


def main() -> int:
    bad = []
    for f, ks in FILES.items():
        bad += check_file(f, ks)
    for b in bad:
        print(b)
    print("ok" if not bad else f"{len(bad)} LDS-DMA hand-off violation(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
