# round-5 GPU step: ragged wgrad GEMM tests, vendor-GEMM reproducer, llama_tiny delayed-DP2 race trace old vs new routing
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_tn" > gpurun_out/r5b_gemm_tests.log 2>&1
timeout -k 10 400 python -u tools/vendor_gemm_repro.py --trials 10 > gpurun_out/r5b_vendor_repro.log 2>&1
export SCALING_AMD_SINGLE_STREAM=0 SCALING_AMD_COMM_DELAY_US=1000 RACE_TRACE_RUNS=3
SCALING_AMD_WGRAD_RAGGED=0 TAG=r5b_old RACE_ARGS="--gpus 2" bash tools/gpu.sh race_trace
SCALING_AMD_WGRAD_RAGGED=1 TAG=r5b_new RACE_ARGS="--gpus 2" bash tools/gpu.sh race_trace
