# round 5 race forensics: does the in-context attention-backward mismatch need the HIP weight-gradient GEMM (LDS-DMA)
# running beside it?  FA_TWICE runs with every wgrad on hipBLASLt vs the default
mkdir -p gpurun_out
summ() {
python - >> gpurun_out/r5z_summary.txt <<'PY'
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
  echo "wgrad on hipBLASLt, set $i" >> gpurun_out/r5z_summary.txt
  SCALING_AMD_WGRAD_HIP=0 SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5z_trace_blas_$i.log 2>&1; summ
  echo "default (HIP wgrad), set $i" >> gpurun_out/r5z_summary.txt
  SCALING_AMD_DEBUG_FA_TWICE=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5z_trace_hip_$i.log 2>&1; summ
done
