# round 5 race forensics: every fused attention backward computed twice in context; mismatch counts in the trace
mkdir -p gpurun_out
for i in 1 2; do
SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5x_trace_twice_$i.log 2>&1
echo "twice $i rc=$?" >> gpurun_out/r5x_summary.txt
python - >> gpurun_out/r5x_summary.txt <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/race_trace/run*.rank*.jsonl")):
    bad = 0
    for line in open(f):
        r = json.loads(line)
        bad += sum(int(v[0] != 0) for n, v in r.get("gtrace", []) if n == "rope_flash.twice_mismatch")
    print(f, "nonzero twice_mismatch entries:", bad)
PY
done
