# race-check forensics (round 5): delayed DP2 multi-stream runs, repeated, with every GEMM on the HIP kernels
# (llama_tiny_r256 + SCALING_AMD_NT_GEMM=1 + SCALING_AMD_DGRAD_WT=all) and with the default vendor GEMMs
set -e
mkdir -p gpurun_out
export SCALING_AMD_NT_GEMM=1 SCALING_AMD_DGRAD_WT=all
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_e1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model llama_tiny_r256 --seq-len 256 --micro-batch 2 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_e1.log 2>&1)
export SCALING_AMD_SINGLE_STREAM=0 SCALING_AMD_COMM_DELAY_US=1000 RACE_TRACE_RUNS=${RACE_TRACE_RUNS:-3}
TAG=e1nt RACE_ARGS="--gpus 2 --model llama_tiny_r256" bash tools/gpu.sh race_trace
unset SCALING_AMD_NT_GEMM SCALING_AMD_DGRAD_WT
TAG=e1vendor RACE_ARGS="--gpus 2 --model llama_tiny_r256" bash tools/gpu.sh race_trace
