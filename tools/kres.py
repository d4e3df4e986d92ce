"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel (VGPR/AGPR/spill/LDS)."""
import re
import subprocess
import sys


def main() -> None:
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-Icsrc/kernels",
                          "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/kres.o"],
                         capture_output=True, text=True).stderr
    cur = None
    rows = {}
    for line in out.splitlines():
        m = re.search(r"remark: (.*?): (.*) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
            rows[cur] = {}
        elif cur:
            rows[cur][k] = v
    for name, r in rows.items():
        if filt in name:
            print(f"{name[:70]:70s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>4} "
                  f"spill {r.get('VGPRs Spill','?'):>4} scratch {r.get('ScratchSize [bytes/lane]','?'):>5} "
                  f"LDS {r.get('LDS Size [bytes/block]','?')} occ {r.get('Occupancy [waves/SIMD]','?')}")


if __name__ == "__main__":
    main()
