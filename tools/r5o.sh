# round 5: race forensics with saved-tensor checksums of the fused rope+flash node (forward vs backward)
set -e
mkdir -p gpurun_out
SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5o_trace_multi.log 2>&1
