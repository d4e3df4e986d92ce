# round-5 GPU step: per-rank shard proxies of BASELINE #3 / #4 (collectives stubbed) + checkpointing A/B + kernel summary
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u bench.py --shard-proxy baseline3 --steps 4 --warmup 2 > gpurun_out/r5d_proxy3.log 2>&1
for ac in disabled every_layer every_layer_save_matmuls; do
  $T 400 python -u bench.py --shard-proxy baseline4 --steps 3 --warmup 1 --activation-checkpointing $ac > gpurun_out/r5d_proxy4_$ac.log 2>&1
done
TAG=r5d_proxy3 PROF_ARGS="--shard-proxy baseline3 --steps 2 --warmup 1" bash tools/gpu.sh prof
