#!/bin/bash
# GPU box: headline bench + kernel profile of a step, activation-checkpointing benches (every_layer and
# every_layer_keep_attention), LoRA bench, graph decode.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r3h}
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --activation-checkpointing every_layer_keep_attention \
    > gpurun_out/bench_ack_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --activation-checkpointing every_layer > gpurun_out/bench_ac_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --lora > gpurun_out/bench_lora_$TAG.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
cd "$R"
python tools/rocpd_step.py /tmp/prof_$TAG/run_results.db > gpurun_out/step_$TAG.md 2>&1 || true
rm -rf /tmp/prof_$TAG
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/decode_$TAG.log 2>&1
