#!/bin/bash
# GPU box (round-2 re-entry): GPU tests + smoke on the rebuilt tree, TunableOp tuning of the micro-batch-8
# shapes (32k-token GEMMs, extends the shipped table), interleaved A/B of mb4 x acc2 vs mb8 x acc1 with the
# extended table, then PMC passes for the weight-gradient GEMM and the attention kernels.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r2i}
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo "tests: $(tail -1 gpurun_out/gpu_tests_$TAG.log)"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  echo "smoke ok"
fi
if [ "${SKIP_TUNE:-0}" != 1 ]; then
  timeout -k 10 700 python -u bench.py --steps 1 --warmup 1 --micro-batch 8 --grad-acc 1 --gemm-tuning tune \
      --gemm-tuning-out "$R/gpurun_out/gemm_tuned_$TAG.csv" > gpurun_out/bench_tune_$TAG.log 2>&1
  cp "$R/gpurun_out/gemm_tuned_$TAG.csv" scaling_amd/tuning/gemm_gfx950.csv
  echo "tuned: $(wc -l < scaling_amd/tuning/gemm_gfx950.csv) lines"
fi
for rep in 1 2; do
  for cfg in "4 2" "8 1"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --micro-batch $1 --grad-acc $2 \
        > gpurun_out/bench_${TAG}_mb$1_acc$2_$rep.log 2>&1
    echo "mb$1 acc$2 rep$rep: $(tail -1 gpurun_out/bench_${TAG}_mb$1_acc$2_$rep.log | cut -c1-200)"
  done
done
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$R/gpurun_out/pmc_gemm1_$TAG" -o a --output-format csv -- python3 "$R/tools/gemm_one.py" 22016 4096 16384 10 \
    > "$R/gpurun_out/pmc_gemm1_$TAG.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d "$R/gpurun_out/pmc_gemm2_$TAG" -o a --output-format csv -- \
    python3 "$R/tools/gemm_one.py" 22016 4096 16384 10 > "$R/gpurun_out/pmc_gemm2_$TAG.log" 2>&1
ITERS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$R/gpurun_out/pmc_attn1_$TAG" -o a --output-format csv -- python3 "$R/tools/attn_only.py" > "$R/gpurun_out/pmc_attn1_$TAG.log" 2>&1
ITERS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d "$R/gpurun_out/pmc_attn2_$TAG" -o a --output-format csv -- python3 "$R/tools/attn_only.py" \
    > "$R/gpurun_out/pmc_attn2_$TAG.log" 2>&1
echo "pmc done"
