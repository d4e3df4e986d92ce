# round 5 race forensics: the attention backward computed three times in context, RoPE folded into the dQ / dK
# epilogues (default) vs plain epilogues + the stand-alone inverse RoPE kernel; 31 steps per run
mkdir -p gpurun_out
summ() {
python - >> gpurun_out/r6h_summary.txt <<'PY'
import json, glob
n = bad = 0
for f in sorted(glob.glob("gpurun_out/race_trace/run*.rank*.jsonl")):
    for line in open(f):
        r = json.loads(line)
        for name, v in r.get("gtrace", []):
            if name == "rope_flash.twice_mismatch":
                n += 1
                bad += int(v[0] != 0)
                if v[0]:
                    print("     ", f, v)
print("   twice-computed attention backwards:", n, "mismatching:", bad)
PY
}
for i in 1 2; do
  for unfold in 0 1; do
    echo "unfold=$unfold, set $i" >> gpurun_out/r6h_summary.txt
    rm -rf gpurun_out/race_trace
    SCALING_AMD_DEBUG_UNFOLD_ROPE=$unfold SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 300 python -u tools/race_trace.py --gpus 2 --steps 30 > gpurun_out/r6h_trace_${unfold}_$i.log 2>&1 || exit 1
    summ
  done
done
