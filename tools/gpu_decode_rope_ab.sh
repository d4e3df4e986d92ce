#!/bin/bash
# GPU box: decode tests with the one-launch norm + q/k/v + RoPE + K/V-append step off (default) and on, then the
# graph-decode latency A/B of it.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-dr}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_e2e.py \
    tests/test_kernels_gpu.py tests/test_inference_module.py -k "decod or generation or graph or flash or gemv or rope or inference" \
    > gpurun_out/dr_tests_$TAG.log 2>&1
SCALING_AMD_DECODE_ROPE_GEMV=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_e2e.py -k "decode or generation" > gpurun_out/dr_tests_rope_$TAG.log 2>&1
for i in 1 2; do
  SCALING_AMD_DECODE_ROPE_GEMV=1 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_rope_${i}_$TAG.log 2>&1
  SCALING_AMD_DECODE_ROPE_GEMV=0 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_norope_${i}_$TAG.log 2>&1
done
