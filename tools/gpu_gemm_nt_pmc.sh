#!/bin/bash
# GPU box: LDS / wait counters of the forward GEMM ring kernel (gemm_nt) vs the wgrad ring kernel at 4096-wide shapes.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$R/gpurun_out/pmc_nt" -o a --output-format csv -- python3 "$R/tools/gemm_nt_one.py" 32768 4096 4096 10 \
    > "$R/gpurun_out/pmc_nt.log" 2>&1
export GEMM_VARIANT=13
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$R/gpurun_out/pmc_tn" -o a --output-format csv -- python3 "$R/tools/gemm_one.py" 4096 4096 32768 10 \
    > "$R/gpurun_out/pmc_tn.log" 2>&1
cd "$R"
python tools/pmc_csv_summary.py gpurun_out/pmc_nt > gpurun_out/pmc_nt.txt 2>&1 || true
python tools/pmc_csv_summary.py gpurun_out/pmc_tn > gpurun_out/pmc_tn.txt 2>&1 || true
