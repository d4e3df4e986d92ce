#!/bin/bash
# GPU box: full GPU suite (incl. multi-rank rehearsal) + smoke + default bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-final}
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
echo "tests: $(tail -1 gpurun_out/gpu_tests_$TAG.log)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
echo "smoke: $(tail -1 gpurun_out/smoke_$TAG.log)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1
echo "bench: $(tail -1 gpurun_out/bench_$TAG.log | cut -c1-260)"
