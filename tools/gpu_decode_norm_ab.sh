#!/bin/bash
# GPU box: norm-prologue GEMV tests + decode GPU tests, then graph-decode latency A/B of the RMSNorm-into-GEMV
# fusion (interleaved runs, one box) and a kernel trace of the fused decode summarised on the box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-dn}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
    -k "gemv or norm or rope_kv" tests/test_gpu_e2e.py > gpurun_out/dn_tests_$TAG.log 2>&1
for i in 1 2; do
  SCALING_AMD_DECODE_NORM_GEMV=1 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_norm_${i}_$TAG.log 2>&1
  SCALING_AMD_DECODE_NORM_GEMV=0 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_nonorm_${i}_$TAG.log 2>&1
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pd_$TAG -o run -- python3 "$R/tools/decode_bench.py" --tokens 32 \
    > "$R/gpurun_out/dec_prof_$TAG.log" 2>&1
cd "$R"
python tools/rocpd_summary.py /tmp/pd_$TAG/run_results.db > gpurun_out/dec_kernels_$TAG.md 2>&1 || true
rm -rf /tmp/pd_$TAG
