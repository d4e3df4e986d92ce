#!/bin/bash
# GPU box: decode kernels + generation tests, graph-decode latency (fused RoPE/cache append + GEMV epilogues) A/B,
# LoRA bench (BASELINE #5 path).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r3d}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "tests/test_kernels_gpu.py::test_rope_kv_append_bit_identical" tests/test_gpu_e2e.py > gpurun_out/dec_tests_$TAG.log 2>&1
for i in 1 2; do
  SCALING_AMD_DECODE_FUSED=1 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_fused_${i}_$TAG.log 2>&1
  SCALING_AMD_DECODE_FUSED=0 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_unfused_${i}_$TAG.log 2>&1
done
timeout -k 10 400 python -u bench.py --lora --steps 5 --warmup 2 > gpurun_out/bench_lora_$TAG.log 2>&1
