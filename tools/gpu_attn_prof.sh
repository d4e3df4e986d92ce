#!/bin/bash
# GPU box: per-kernel times (rocprofv3 kernel stats) of the attention-only driver for the base and new builds
# (abso/*.so), then two PMC passes on the new build.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SO=$(ls scaling_amd/_C.cpython-*.so)
cd /tmp
export TMPDIR=/tmp
for b in base new; do
  cp "$R/abso/${b}_C.so" "$R/$SO"
  ITERS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/attnprof_$b" -o run -- python3 "$R/tools/attn_only.py" \
      > "$R/gpurun_out/attnprof_$b.log" 2>&1
done
ITERS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
    -d "$R/gpurun_out/attnpmc1" -o a --output-format csv -- python3 "$R/tools/attn_only.py" > "$R/gpurun_out/attnpmc1.log" 2>&1
ITERS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d "$R/gpurun_out/attnpmc2" -o a --output-format csv -- python3 "$R/tools/attn_only.py" \
    > "$R/gpurun_out/attnpmc2.log" 2>&1
