#!/bin/bash
# GPU box: gemm_tn correctness (all variants incl. 8), then variant 2 vs 8 at the 7B wgrad shapes (interleaved).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-g8}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn" -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_gemm_$TAG.log 2>&1
timeout -k 10 400 python -u tools/gemm_bench.py --tokens 32768 --variants ${VARIANTS:-2,8,9} --iters 10 --rounds 3 > gpurun_out/gemm_bench_$TAG.log 2>&1
