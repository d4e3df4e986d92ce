#!/bin/bash
# GPU box: full GPU suite + smoke, default 1-GPU bench twice, LoRA bench (fused base weights re-homed), decode
# bench, and a rocprofv3 kernel profile of the default bench step.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r2n}
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
echo "tests: $(tail -1 gpurun_out/gpu_tests_$TAG.log)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
echo "smoke ok"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_${TAG}_$rep.log 2>&1
  echo "bench $rep: $(tail -1 gpurun_out/bench_${TAG}_$rep.log | cut -c1-260)"
done
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --lora > gpurun_out/bench_${TAG}_lora.log 2>&1
echo "lora: $(tail -1 gpurun_out/bench_${TAG}_lora.log | cut -c1-260)"
timeout -k 10 400 python -u tools/decode_bench.py --model llama2_7b > gpurun_out/decode_7b_$TAG.log 2>&1
echo "decode: $(tail -1 gpurun_out/decode_7b_$TAG.log)"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
echo "profile done"
