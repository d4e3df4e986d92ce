#!/bin/bash
# GPU box: paired, software-pipelined dK/dV (SCALING_AMD_FA_BWD_PAIR=1): attention tests, then timing A/B.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-pair}
SCALING_AMD_FA_BWD_PAIR=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_production.py -m gpu \
    -x -q --timeout 120 --timeout-method thread -k "attention or flash" > gpurun_out/attn_pair_tests_$TAG.log 2>&1
for rep in 1 2; do
  for pr in 0 1; do
    echo "== pair=$pr rep $rep" >> gpurun_out/attn_pair_ab_$TAG.log
    SCALING_AMD_FA_BWD_PAIR=$pr ITERS=10 timeout -k 10 120 python -u tools/attn_only.py >> gpurun_out/attn_pair_ab_$TAG.log 2>&1
  done
done
