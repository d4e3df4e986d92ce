#!/bin/bash
# GPU box: GEMV kernel tests, graph-decode tests, decode latency bench (1B, 7B).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r2m}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "gemv or graph_decode or cached_generation" > gpurun_out/tests_$TAG.log 2>&1
echo "tests: $(tail -1 gpurun_out/tests_$TAG.log)"
timeout -k 10 300 python -u tools/decode_bench.py --model llama_1b > gpurun_out/decode_1b_$TAG.log 2>&1
echo "1b: $(tail -1 gpurun_out/decode_1b_$TAG.log)"
timeout -k 10 400 python -u tools/decode_bench.py --model llama2_7b > gpurun_out/decode_7b_$TAG.log 2>&1
echo "7b: $(tail -1 gpurun_out/decode_7b_$TAG.log)"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_dec_$TAG" -o run -- python3 "$R/tools/decode_bench.py" \
    --model llama2_7b --tokens 16 > "$R/gpurun_out/decode_prof_$TAG.log" 2>&1
echo "profile done"
