#!/bin/bash
# GPU box: re-tune every hipBLASLt shape of the default bench from scratch (validator-only start file), then A/B
# the bench with the shipped table vs the fresh one on the same box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
grep "^Validator" scaling_amd/tuning/gemm_gfx950.csv > gpurun_out/gemm_fresh.csv
timeout -k 10 1000 python -u bench.py --steps 1 --warmup 1 --gemm-tuning tune --gemm-tuning-out gpurun_out/gemm_fresh.csv \
    > gpurun_out/fresh_tune.log 2>&1
echo "fresh rows: $(grep -vc Validator gpurun_out/gemm_fresh.csv)"
cp scaling_amd/tuning/gemm_gfx950.csv gpurun_out/gemm_shipped.csv
for rep in 1 2; do
  cp gpurun_out/gemm_shipped.csv scaling_amd/tuning/gemm_gfx950.csv
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/tune_ab_shipped_$rep.log 2>&1
  echo "shipped $rep: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tune_ab_shipped_$rep.log)"
  cp gpurun_out/gemm_fresh.csv scaling_amd/tuning/gemm_gfx950.csv
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/tune_ab_fresh_$rep.log 2>&1
  echo "fresh $rep: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tune_ab_fresh_$rep.log)"
done
