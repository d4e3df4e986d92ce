# round 5 race forensics: attention backward with a 48-cycle pad between its last MFMAs and the epilogue reads
mkdir -p gpurun_out
summ() {
python - >> gpurun_out/r6j_summary.txt <<'PY'
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
for i in 1 2 3; do
  for pad in 0 1; do
    echo "pad=$pad, set $i" >> gpurun_out/r6j_summary.txt
    rm -rf gpurun_out/race_trace
    SCALING_AMD_EXT_SO=$( [ $pad = 1 ] && echo $PWD/variants/bwdpad.so ) SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 300 python -u tools/race_trace.py --gpus 2 --steps 30 > gpurun_out/r6j_trace_${pad}_$i.log 2>&1 || exit 1
    summ
  done
done
