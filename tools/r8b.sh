# round 5 re-entry: headline bench (20 + 5, the driver's protocol) + 3-step kernel profile
mkdir -p gpurun_out
BENCH_ARGS="--steps 20 --warmup 5" TAG=r8b bash tools/gpu.sh bench prof || exit 1
