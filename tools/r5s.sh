set -e
mkdir -p gpurun_out
SCALING_AMD_BENCH_NORMS=1 timeout -k 10 300 python -u bench.py --shard-proxy baseline3 --num-layers 16 --steps 1 --warmup 0 > gpurun_out/r5s_proxy_norms.log 2>&1 || true
SCALING_AMD_BENCH_NORMS=1 SCALING_AMD_SP_OVERLAP=0 SCALING_AMD_DEFER_RESIDUAL=0 timeout -k 10 300 python -u bench.py --shard-proxy baseline3 --num-layers 16 --steps 1 --warmup 0 --tp-comm-chunks 1 > gpurun_out/r5s_proxy_norms_plain.log 2>&1 || true
