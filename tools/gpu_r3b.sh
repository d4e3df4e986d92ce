#!/bin/bash
# GPU box: (1) where the activation-checkpointed 7B step idles (full 32 layers, HIP API + kernel trace, summarised
# on the box), (2) keep-attention AC bench with expandable allocator segments, (3) headline bench + kernel profile,
# (4) graph-decode latency with the fused GEMV epilogues.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r3b}
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d /tmp/tr_$TAG -o t -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --activation-checkpointing every_layer_keep_attention \
    > "$R/gpurun_out/trace_ac_$TAG.log" 2>&1
cd "$R"
python tools/gap_summary.py /tmp/tr_$TAG 200 > gpurun_out/gaps_ac32_$TAG.txt 2>&1 || true
python tools/sync_trace_summary.py /tmp/tr_$TAG > gpurun_out/sync_ac32_$TAG.txt 2>&1 || true
rm -rf /tmp/tr_$TAG
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 \
    --activation-checkpointing every_layer_keep_attention > gpurun_out/bench_ack_exp_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
cd "$R"
python tools/rocpd_step.py /tmp/prof_$TAG/run_results.db > gpurun_out/step_$TAG.md 2>&1 || true
rm -rf /tmp/prof_$TAG
timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/decode_$TAG.log 2>&1
