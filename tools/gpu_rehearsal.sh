#!/bin/bash
# GPU box: multi-rank rehearsal (bench.py ranks sharing the GPU over gloo) + the rest of the GPU suite selection.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-reh}
timeout -k 10 900 python -u -m pytest tests/test_gpu_rehearsal.py ${EXTRA_TESTS:-} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_rehearsal_$TAG.log 2>&1
echo "rehearsal: $(tail -1 gpurun_out/gpu_rehearsal_$TAG.log)"
