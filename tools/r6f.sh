# round 5 race forensics: rehearsal ranks on disjoint CU halves (HSA_CU_MASK) -- does the in-context attention-backward
# mismatch need another process's waves on the same CUs?
mkdir -p gpurun_out
summ() {
python - >> gpurun_out/r6f_summary.txt <<'PY'
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
for i in 1 2 3 4; do
  echo "CU split, set $i" >> gpurun_out/r6f_summary.txt
  SCALING_AMD_REHEARSAL_CU_SPLIT=256 SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r6f_trace_split_$i.log 2>&1; summ
  grep -v amdgpu gpurun_out/r6f_trace_split_$i.log | grep "vs run 0" | grep -vc identical >> gpurun_out/r6f_summary.txt
done
