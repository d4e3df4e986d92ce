#!/bin/bash
# GPU box: 1-GPU headline bench, rocprofv3 kernel stats of 3 steps.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1 )
