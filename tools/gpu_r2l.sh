#!/bin/bash
# GPU box: graph-captured decoding tests + the decode latency bench (small model, then the 7B shape).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r2l}
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "graph_decode or cached_generation or lazy" > gpurun_out/tests_$TAG.log 2>&1
echo "tests: $(tail -1 gpurun_out/tests_$TAG.log)"
timeout -k 10 300 python -u tools/decode_bench.py --model llama_1b > gpurun_out/decode_1b_$TAG.log 2>&1
echo "1b: $(tail -1 gpurun_out/decode_1b_$TAG.log)"
timeout -k 10 400 python -u tools/decode_bench.py --model llama2_7b > gpurun_out/decode_7b_$TAG.log 2>&1
echo "7b: $(tail -1 gpurun_out/decode_7b_$TAG.log)"
