#!/bin/bash
# Emulated-collective check of the per-rank proxy: stub vs emulate (link efficiency forced low) on the test's small
# shape, plus a kernel trace of the emulated run (xgmi_emu_kernel launches and their durations).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/emu_dbg
ARGS="--model llama_tiny_r256 --seq-len 256 --micro-batch 8 --steps ${STEPS:-6} --warmup 2 --shard-proxy baseline3"
timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/emu_dbg/stub.log 2>&1
SCALING_AMD_PROXY_COMM_EFF=0.00065 timeout -k 10 200 python -u bench.py $ARGS --proxy-comm emulate > gpurun_out/emu_dbg/emu.log 2>&1
cd /tmp && export TMPDIR=/tmp
SCALING_AMD_PROXY_COMM_EFF=0.00065 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/emu_dbg/prof" -o run -- \
    python3 -u "$R/bench.py" $ARGS --proxy-comm emulate > "$R/gpurun_out/emu_dbg/prof.log" 2>&1
