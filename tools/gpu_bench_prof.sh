#!/bin/bash
# GPU box: gpu tests, smoke, 1-GPU bench and a rocprofv3 kernel-stats profile of 3 bench steps.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
