#!/bin/bash
# GPU box: attention A/B between two builds of the extension (abso/base_C.so vs abso/new_C.so, interleaved twice),
# then the attention kernel tests on the new build.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SO=$(ls scaling_amd/_C.cpython-*.so)
for rep in 1 2; do
  for b in base new; do
    cp abso/${b}_C.so "$SO"
    echo "== $b $rep" >> gpurun_out/attn_ab.log
    ITERS=10 timeout -k 10 120 python -u tools/attn_only.py >> gpurun_out/attn_ab.log 2>&1
  done
done
cp abso/new_C.so "$SO"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_production.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "attention or dropout or flash or decode" > gpurun_out/attn_ab_tests.log 2>&1
