# round 5: attention reproducibility under load, strided-bmm probe, DP2 race traces, shard proxies
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "flash or swiglu" > gpurun_out/r5h_kernel_tests.log 2>&1
$T 120 python -u tools/attn_only.py > gpurun_out/r5h_attn.log 2>&1
$T 300 python -u tools/attn_repro.py --trials 10 > gpurun_out/r5h_attn_repro.log 2>&1

SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=3 $T 400 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5h_trace_multi.log 2>&1
RACE_TRACE_RUNS=3 $T 400 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5h_trace_single.log 2>&1


