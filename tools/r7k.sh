# round 5: stall counters (wave-cycles waiting / issue-waiting / active by type) for the attention kernels and the wgrad
# GEMM, one rocprofv3 --pmc pass each (8 SQ + 1 GRBM counters)
R=$(pwd)
mkdir -p gpurun_out
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
(cd /tmp && export TMPDIR=/tmp && ITERS=2 timeout -s KILL 150 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_attn -o a --output-format csv -- python3 $R/tools/attn_only.py > $R/gpurun_out/pmc_attn.log 2>&1) || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_wgrad -o a --output-format csv -- python3 $R/tools/wgrad_bench.py --rounds 1 --iters 2 > $R/gpurun_out/pmc_wgrad.log 2>&1) || exit 1
