#!/bin/bash
# GPU box: attention kernel tests + timing + rocprofv3 kernel stats (outputs under gpurun_out/).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "attention or dropout" > gpurun_out/gpu_tests_attn.log 2>&1
ITERS=10 timeout -k 10 120 python -u tools/attn_only.py > gpurun_out/attn.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_attn" -o run -- python3 "$R/tools/attn_only.py" \
    > "$R/gpurun_out/attn_prof.log" 2>&1
