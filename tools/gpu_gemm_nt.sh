#!/bin/bash
# GPU box: gemm_nt correctness, then the forward / dgrad GEMM shapes vs hipBLASLt (TunableOp table).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-nt}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_nt" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tests_gemm_nt_$TAG.log 2>&1
timeout -k 10 600 python -u tools/gemm_nt_bench.py > gpurun_out/gemm_nt_bench_$TAG.log 2>&1
