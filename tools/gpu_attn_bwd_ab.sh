#!/bin/bash
# GPU box: backward kernel variants (SCALING_AMD_FA_BWD_OCC = 1/2 x SCALING_AMD_FA_BWD_ADMA = 0/1): attention tests for
# each new combination, then fwd/bwd timing interleaved twice.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-bwd}
for combo in "2 1" "1 0" "1 1"; do
  set -- $combo
  SCALING_AMD_FA_BWD_OCC=$1 SCALING_AMD_FA_BWD_ADMA=$2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py \
      tests/test_gpu_production.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or flash" \
      >> gpurun_out/attn_bwd_tests_$TAG.log 2>&1
  echo "== combo occ=$1 adma=$2 ok" >> gpurun_out/attn_bwd_tests_$TAG.log
done
SCALING_AMD_FA_FWD_ADMA=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_production.py -m gpu \
    -x -q --timeout 120 --timeout-method thread -k "attention or flash" >> gpurun_out/attn_bwd_tests_$TAG.log 2>&1
echo "== fwd adma ok" >> gpurun_out/attn_bwd_tests_$TAG.log
for rep in 1 2; do
  for combo in "2 0" "2 1" "1 0" "1 1"; do
    set -- $combo
    echo "== occ=$1 adma=$2 (fwd adma=$2) rep $rep" >> gpurun_out/attn_bwd_ab_$TAG.log
    SCALING_AMD_FA_FWD_ADMA=$2 SCALING_AMD_FA_BWD_OCC=$1 SCALING_AMD_FA_BWD_ADMA=$2 ITERS=10 timeout -k 10 120 \
        python -u tools/attn_only.py >> gpurun_out/attn_bwd_ab_$TAG.log 2>&1
  done
done
