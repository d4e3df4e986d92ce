#!/bin/bash
# GPU box: HIP API trace of a short training run: which synchronizing HIP calls happen per step.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$R/gpurun_out/synctrace" -o t -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --num-layers 4 > "$R/gpurun_out/synctrace.log" 2>&1
cd "$R"
python tools/sync_trace_summary.py gpurun_out/synctrace > gpurun_out/synctrace.txt
cat gpurun_out/synctrace.txt
