# round 5 race forensics: checksum of the attention backward's output right after the kernel; device syncs around it
mkdir -p gpurun_out
SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=5 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5w_trace_multi.log 2>&1
echo "multi rc=$?" >> gpurun_out/r5w_summary.txt
SCALING_AMD_DEBUG_SYNC_FA=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=5 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5w_trace_syncfa.log 2>&1
echo "syncfa rc=$?" >> gpurun_out/r5w_summary.txt
