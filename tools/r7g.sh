# round 5 validation of the tree: whole GPU suite, smoke, 1-GPU bench (driver-like 20 + 5), step profile
mkdir -p gpurun_out
TAG=r7g bash tools/gpu.sh tests smoke || exit 1
BENCH_ARGS="--steps 20 --warmup 5" TAG=r7g bash tools/gpu.sh bench prof || exit 1
