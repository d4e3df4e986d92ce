# round 5 final-tree validation: whole GPU suite, smoke, headline bench (20 + 5), step profile
mkdir -p gpurun_out
TAG=r7u bash tools/gpu.sh tests smoke || exit 1
BENCH_ARGS="--steps 20 --warmup 5" TAG=r7u bash tools/gpu.sh bench prof || exit 1
