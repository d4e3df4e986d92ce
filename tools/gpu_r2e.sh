#!/bin/bash
# GPU box: default bench (mb4 x acc2) with peak memory, an mb8 x acc1 probe (may OOM: not fatal), the small-GPT
# transformer example (BASELINE config #2) through the runner, and a rocprofv3 profile of the default bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --micro-batch 8 --grad-acc 1 > gpurun_out/bench_${TAG}_mb8.log 2>&1 || echo "mb8 failed"
tail -1 gpurun_out/bench_${TAG}_mb8.log | cut -c1-200
timeout -k 10 120 python -u examples/transformer_example/make_synthetic_data.py examples/transformer_example/data/data \
    > gpurun_out/example_$TAG.log 2>&1
timeout -k 10 300 python -u -m examples.transformer_example.run examples/transformer_example/config.yml >> gpurun_out/example_$TAG.log 2>&1
tail -3 gpurun_out/example_$TAG.log | cut -c1-300
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
