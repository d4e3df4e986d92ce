# round 5 final evidence on one box: GPU suite, smoke, headline bench (driver protocol 20 + 5), step profile, BASELINE
# #3/#4 per-rank proxies, LoRA, decode
mkdir -p gpurun_out
TAG=r7n bash tools/gpu.sh tests smoke || exit 1
BENCH_ARGS="--steps 20 --warmup 5" TAG=r7n bash tools/gpu.sh bench prof || exit 1
BENCH_ARGS="--shard-proxy baseline3 --steps 5 --warmup 2" TAG=r7n_b3 bash tools/gpu.sh bench || exit 1
BENCH_ARGS="--shard-proxy baseline4 --steps 5 --warmup 2" TAG=r7n_b4 bash tools/gpu.sh bench || exit 1
BENCH_ARGS="--lora --steps 5 --warmup 2" TAG=r7n_lora bash tools/gpu.sh bench || exit 1
TAG=r7n bash tools/gpu.sh decode || exit 1
