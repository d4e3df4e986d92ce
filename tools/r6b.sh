# round 5 race forensics: twice-computed attention backward with every side stream folded (single) vs multi
mkdir -p gpurun_out
summ() {
python - >> gpurun_out/r6b_summary.txt <<'PY'
import json, glob
n = bad = 0
for f in sorted(glob.glob("gpurun_out/race_trace/run*.rank*.jsonl")):
    for line in open(f):
        r = json.loads(line)
        for name, v in r.get("gtrace", []):
            if name == "rope_flash.twice_mismatch":
                n += 1
                bad += int(v[0] != 0)
print("   twice-computed attention backwards:", n, "mismatching:", bad)
PY
}
for i in 1 2 3; do
  for m in 1 0; do
    echo "SINGLE_STREAM=$m set $i" >> gpurun_out/r6b_summary.txt
    SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=$m RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r6b_trace_s${m}_$i.log 2>&1; summ
  done
done
