#!/bin/bash
# GPU box: PMC counters (MFMA busy, wave cycles, waits, clock) of the wgrad GEMM variants at the gate/up shape.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-pmc2}
SHAPE=${SHAPE:-"22016 4096 32768"}
cd /tmp
export TMPDIR=/tmp
for V in ${VARIANTS:-2 10}; do
  export GEMM_VARIANT=$V
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
      -d "$R/gpurun_out/pmc_${TAG}_v$V" -o a --output-format csv -- python3 "$R/tools/gemm_one.py" $SHAPE 10 \
      > "$R/gpurun_out/pmc_${TAG}_v$V.log" 2>&1
done
cd "$R"
for V in ${VARIANTS:-2 10}; do python tools/pmc_csv_summary.py gpurun_out/pmc_${TAG}_v$V > gpurun_out/pmc_${TAG}_v$V.txt 2>&1 || true; done
