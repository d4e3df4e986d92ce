#!/bin/bash
# GPU box: selective recompute (every_layer_save_matmuls): checkpointing GPU tests, then the 7B AC bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-acsm}
timeout -k 10 600 python -u -m pytest tests/test_gpu_rehearsal.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "checkpointing" > gpurun_out/ac_sm_tests_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --activation-checkpointing every_layer_save_matmuls \
    > gpurun_out/bench_acsm_$TAG.log 2>&1
