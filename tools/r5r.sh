# round 5: rope-fused attention reproducibility under load; race trace with cos/sin/cu in the saved-tensor record;
# proxy grad-magnitude debug at 16 layers
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_repro.py --trials 10 > gpurun_out/r5r_attn_repro_rope.log 2>&1
SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=4 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5r_trace_multi.log 2>&1
SCALING_AMD_BENCH_NORMS=1 timeout -k 10 300 python -u bench.py --shard-proxy baseline3 --num-layers 16 --steps 1 --warmup 0 > gpurun_out/r5r_proxy_norms.log 2>&1 || true
