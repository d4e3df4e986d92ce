# round 5 race forensics: where the twice-computed fused attention backward differs (q / k / v slice, first indices)
mkdir -p gpurun_out
for i in 1 2 3; do
SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5y_trace_twice_$i.log 2>&1
python - >> gpurun_out/r5y_summary.txt <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/race_trace/run*.rank*.jsonl")):
    for line in open(f):
        r = json.loads(line)
        for n, v in r.get("gtrace", []):
            if n == "rope_flash.twice_mismatch" and v[0] != 0:
                print(f, "step", r["step"], "total/dq/dk/dv", v[:4], "first flat idx", v[4:-1], "row len", v[-1])
PY
done
