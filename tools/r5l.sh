# round 5: strided-bmm probe, DP2 race traces (multi-stream and single-stream, 3 runs each), BASELINE #3/#4 proxies
set -e
mkdir -p gpurun_out
T="timeout -k 10"

SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=3 $T 400 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5l_trace_multi.log 2>&1
RACE_TRACE_RUNS=3 $T 400 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5l_trace_single.log 2>&1
bash tools/r5d.sh
