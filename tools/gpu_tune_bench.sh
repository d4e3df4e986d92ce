#!/bin/bash
# GPU box: kernel tests for a change, GEMM re-tuning of the 7B step (TunableOp), then the 1-GPU bench with
# the new table and a rocprofv3 kernel-stats profile.  Outputs under gpurun_out/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS ${TESTK:+-k "$TESTK"} -m gpu -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/tests_$TAG.log 2>&1
fi
if [ "$TUNE" = "1" ]; then
  timeout -k 10 700 python -u bench.py --steps 1 --warmup 1 --gemm-tuning tune \
      --gemm-tuning-out "$R/gpurun_out/gemm_tuned_$TAG.csv" > gpurun_out/bench_tune_$TAG.log 2>&1
  cp "$R/gpurun_out/gemm_tuned_$TAG.csv" scaling_amd/tuning/gemm_gfx950.csv
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
