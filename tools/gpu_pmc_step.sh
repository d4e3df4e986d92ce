#!/bin/bash
# GPU box: PMC counters of every kernel of a 4-layer 7B-width training step (two passes: SQ/GRBM, then HBM fetch).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp
export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 1 --num-layers 4"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$R/gpurun_out/pmc_step_sq" -o a --output-format csv -- python3 $B > "$R/gpurun_out/pmc_step_sq.log" 2>&1
echo "pass 1 done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
    -d "$R/gpurun_out/pmc_step_hbm" -o a --output-format csv -- python3 $B > "$R/gpurun_out/pmc_step_hbm.log" 2>&1
echo "pass 2 done"
cd "$R"
python tools/pmc_csv_summary.py gpurun_out/pmc_step_sq > gpurun_out/pmc_step_sq.txt
python tools/pmc_csv_summary.py gpurun_out/pmc_step_hbm > gpurun_out/pmc_step_hbm.txt
head -40 gpurun_out/pmc_step_sq.txt
