#!/bin/bash
# GPU box: gemm_tn correctness for the pipeline variants, then the 7B-shape wgrad benchmark A/B in one process.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn" -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_gemm_$TAG.log 2>&1
timeout -k 10 300 python -u tools/gemm_bench.py --variants ${VARIANTS:-2,4,2,4} --iters 30 > gpurun_out/gemm_bench_$TAG.log 2>&1
