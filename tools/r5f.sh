set -e
mkdir -p gpurun_out
export SCALING_AMD_SINGLE_STREAM=0 SCALING_AMD_COMM_DELAY_US=1000 RACE_TRACE_RUNS=4
TAG=r5f RACE_ARGS="--gpus 2" bash tools/gpu.sh race_trace
unset SCALING_AMD_SINGLE_STREAM SCALING_AMD_COMM_DELAY_US RACE_TRACE_RUNS
bash tools/r5d.sh
bash tools/r5e.sh
