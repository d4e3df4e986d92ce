#!/bin/bash
# GPU box: keep-attention checkpointing test + decode epilogue tests, 7B bench with per-layer checkpointing (plain vs
# keep-attention), HIP API trace of a checkpointed 4-layer run (host gaps), kernel profile of the keep-attention
# step.  Raw traces are summarised on the box and deleted (gpurun copies back at most 64 MiB).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-ac}
timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread \
    "tests/test_gpu_rehearsal.py::test_keep_attention_checkpointing_gpu" \
    "tests/test_kernels_gpu.py::test_gemv_epilogues_bit_identical" \
    tests/test_gpu_e2e.py > gpurun_out/ac_test_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --activation-checkpointing every_layer > gpurun_out/bench_ac_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --activation-checkpointing every_layer_keep_attention > gpurun_out/bench_ack_$TAG.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d /tmp/synctrace_$TAG -o t -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --num-layers 4 --activation-checkpointing every_layer_keep_attention \
    > "$R/gpurun_out/synctrace_$TAG.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python3 "$R/bench.py" \
    --steps 3 --warmup 1 --activation-checkpointing every_layer_keep_attention > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
cd "$R"
python tools/sync_trace_summary.py /tmp/synctrace_$TAG > gpurun_out/synctrace_$TAG.txt 2>&1 || true
python tools/gap_summary.py /tmp/synctrace_$TAG 50 > gpurun_out/gaps_$TAG.txt 2>&1 || true
python tools/rocpd_step.py /tmp/prof_$TAG/run_results.db > gpurun_out/step_$TAG.md 2>&1 || true
