#!/bin/bash
# GPU box: TunableOp tuning of the 7B step at micro-batch 4 (extends the shipped table), then an interleaved
# A/B of mb2xacc4 vs mb4xacc2 with the extended table.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
timeout -k 10 700 python -u bench.py --steps 1 --warmup 1 --micro-batch 4 --grad-acc 2 --gemm-tuning tune \
    --gemm-tuning-out "$R/gpurun_out/gemm_tuned_$TAG.csv" > gpurun_out/bench_tune_$TAG.log 2>&1
cp "$R/gpurun_out/gemm_tuned_$TAG.csv" scaling_amd/tuning/gemm_gfx950.csv
bash tools/gpu_bench_batch.sh
