# round-5 GPU step: v3 attention forward (asm DMA, VGPR-form S) tests + timing; llama_tiny delayed-DP2 grad trace
set -e
mkdir -p gpurun_out
SCALING_AMD_FA_FWD_V3=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "flash_attention" > gpurun_out/r5c_v3_tests.log 2>&1
SCALING_AMD_FA_FWD_V3=1 timeout -k 10 120 python -u tools/attn_only.py > gpurun_out/r5c_v3_attn.log 2>&1
timeout -k 10 120 python -u tools/attn_only.py > gpurun_out/r5c_v2_attn.log 2>&1
export SCALING_AMD_SINGLE_STREAM=0 SCALING_AMD_COMM_DELAY_US=1000 RACE_TRACE_RUNS=4
TAG=r5c RACE_ARGS="--gpus 2" bash tools/gpu.sh race_trace
