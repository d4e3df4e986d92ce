#!/bin/bash
# GPU box: kernel + e2e GPU tests (one pytest process), then the wgrad GEMM variant A/B benchmark.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_gpu_e2e.py} -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
if [ -n "$VARIANTS" ]; then
  timeout -k 10 300 python -u tools/gemm_bench.py --variants "$VARIANTS" --iters 30 > gpurun_out/gemm_bench_$TAG.log 2>&1
fi
