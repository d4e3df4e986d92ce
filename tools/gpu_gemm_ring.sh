#!/bin/bash
# GPU box: gemm_tn correctness (all variants), determinism stress, ring-kernel stamps, variants A/B at the 7B shapes.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-ring}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tests_gemm_$TAG.log 2>&1
for V in ${RVARIANTS:-9 10 11}; do
  timeout -k 10 300 python -u tools/gemm_repeat_check.py $V 30 >> gpurun_out/repeat_$TAG.log 2>&1
done
for V in ${TVARIANTS:-9 10}; do
  GEMM_VARIANT=$V timeout -k 10 120 python -u tools/gemm_ring_timing.py > gpurun_out/ring_timing_${TAG}_v$V.log 2>&1
done
timeout -k 10 600 python -u tools/gemm_bench.py --tokens 32768 --variants ${VARIANTS:-2,9,10,11} --iters 10 --rounds 3 \
    > gpurun_out/gemm_bench_$TAG.log 2>&1
