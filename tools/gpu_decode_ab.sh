#!/bin/bash
# GPU box: graph-decode latency A/B of the fused decode GEMV epilogues (interleaved runs, one box), then a kernel
# trace of the fused decode summarised on the box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-dec}
for i in 1 2; do
  SCALING_AMD_DECODE_FUSED=1 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_fused_${i}_$TAG.log 2>&1
  SCALING_AMD_DECODE_FUSED=0 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_unfused_${i}_$TAG.log 2>&1
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pd_$TAG -o run -- python3 "$R/tools/decode_bench.py" --tokens 32 \
    > "$R/gpurun_out/dec_prof_$TAG.log" 2>&1
cd "$R"
python tools/rocpd_summary.py /tmp/pd_$TAG/run_results.db > gpurun_out/dec_kernels_$TAG.md 2>&1 || true
rm -rf /tmp/pd_$TAG
