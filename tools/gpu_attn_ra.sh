#!/bin/bash
# GPU box: read-ahead variants (SCALING_AMD_FA_FWD_RA=1 forward, SCALING_AMD_FA_BWD_RA=1 dQ): attention tests, then
# timing A/B interleaved three times.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-ra}
SCALING_AMD_FA_FWD_RA=1 SCALING_AMD_FA_BWD_RA=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py \
    tests/test_gpu_production.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or flash" \
    > gpurun_out/attn_ra_tests_$TAG.log 2>&1
for rep in 1 2 3; do
  for ra in 0 1; do
    echo "== ra=$ra rep $rep" >> gpurun_out/attn_ra_ab_$TAG.log
    SCALING_AMD_FA_FWD_RA=$ra SCALING_AMD_FA_BWD_RA=$ra ITERS=20 timeout -k 10 120 python -u tools/attn_only.py \
        >> gpurun_out/attn_ra_ab_$TAG.log 2>&1
  done
done
