"""Per-kernel PMC summary from a rocprofv3 rocpd database (counters averaged per dispatch)."""
import re
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for name, did, cn, v in c.execute("select name, dispatch_id, counter_name, counter_value from pmc_events"):
    if pat not in name:
        continue
    k = re.sub(r"\(.*", "", name).replace("void ", "")[:60]
    agg[k][cn] += v
    disp[k].add(did)
for k, d in agg.items():
    n = len(disp[k])
    print(k, "dispatches", n)
    print("   ", {cn: round(v / n) for cn, v in sorted(d.items())})
    if d.get("SQ_INSTS_MFMA"):
        print("    VALU/MFMA %.2f  LDS/MFMA %.2f  WAIT_INST_ANY/WAVE_CYCLES %.3f" % (
            d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"], d["SQ_INSTS_LDS"] / d["SQ_INSTS_MFMA"],
            d["SQ_WAIT_INST_ANY"] / max(1, d["SQ_WAVE_CYCLES"])))
