#!/bin/bash
# GPU box: wgrad GEMM variant A/B (interleaved rounds, accumulate mode as in the model), then the kernel tests.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 400 python -u tools/gemm_bench.py --variants "${VARIANTS:-2,5}" --iters 20 --rounds 5 > gpurun_out/gemm_ab_$TAG.log 2>&1
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS ${TESTK:+-k "$TESTK"} -m gpu -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/tests_$TAG.log 2>&1
fi
