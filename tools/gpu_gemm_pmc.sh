#!/bin/bash
# GPU box: per-phase stamps of the wgrad GEMM (variant 2) and PMC counters of variants 2 and 5 at the gate/up shape.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-pmc}
SHAPE=${SHAPE:-"22016 4096 16384"}
timeout -k 10 120 python -u tools/gemm_timing.py $SHAPE > gpurun_out/gemm_timing_$TAG.log 2>&1
cd /tmp
export TMPDIR=/tmp
for V in ${VARIANTS:-2 5}; do
  export GEMM_VARIANT=$V
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT \
      -d "$R/gpurun_out/pmc_${TAG}_v$V" -o a --output-format csv -- python3 "$R/tools/gemm_one.py" $SHAPE 10 \
      > "$R/gpurun_out/pmc_${TAG}_v$V.log" 2>&1
done
