# round 5 race forensics: CU-split vs shared CUs, interleaved, 8 runs per set (128 twice-computed backwards per set)
mkdir -p gpurun_out
summ() {
python - >> gpurun_out/r6g_summary.txt <<'PY'
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
for i in 1 2 3 4; do
  for split in 256 0; do
    echo "CU split=$split, set $i" >> gpurun_out/r6g_summary.txt
    rm -rf gpurun_out/race_trace
    SCALING_AMD_REHEARSAL_CU_SPLIT=$split SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=8 timeout -k 10 300 python -u tools/race_trace.py --gpus 2 > gpurun_out/r6g_trace_${split}_$i.log 2>&1 || exit 1
    summ
  done
done
