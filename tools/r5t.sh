# round 5: 7B headline bench + rocprof step breakdown with the round-5 step changes
set -e
mkdir -p gpurun_out
TAG=r5t BENCH_ARGS="--steps 10 --warmup 3" bash tools/gpu.sh bench
TAG=r5t bash tools/gpu.sh prof
