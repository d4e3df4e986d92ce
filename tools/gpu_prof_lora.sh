#!/bin/bash
# GPU box: rocprofv3 kernel profile of the LoRA bench step (BASELINE #5 shape on one GPU).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-lora}
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --lora ${EXTRA:-} \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
cd "$R"
python tools/rocpd_step.py gpurun_out/prof_$TAG/run_results.db > gpurun_out/step_$TAG.md
head -30 gpurun_out/step_$TAG.md
