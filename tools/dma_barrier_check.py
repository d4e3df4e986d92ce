"""Static check of the LDS-DMA hand-off rule in the attention kernels (the race the round-5 gradient trace found).

Every ``s_barrier`` after which waves read tiles that OTHER waves staged by LDS-DMA must be preceded, in each wave, by
an ``s_waitcnt vmcnt(0)`` with no LDS-DMA issue in between (``flash_attn.h: dma_barrier``).  Compiles the kernel files
to gfx950 assembly (the extension build's flags) and walks back from every barrier of the listed kernels.

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


def main() -> int:
    bad = []
    for f, ks in FILES.items():
        bad += check_file(f, ks)
    for b in bad:
        print(b)
    print("ok" if not bad else f"{len(bad)} barrier(s) without a DMA-retiring wait")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
