#!/bin/bash
# GPU box: attention A/B (abso/base_C.so vs abso/new_C.so, interleaved) + attention tests on the new build,
# the default 1-GPU bench, a rocprofv3 kernel profile of it, and 1-GPU numbers for the activation-checkpointing
# and LoRA paths (BASELINE configs #4/#5 run them at 8 GPUs; here the 7B shape on one).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r2j}
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
SO=$(ls scaling_amd/_C.cpython-*.so)
if [ -f abso/new_C.so ]; then
  for rep in 1 2; do
    for b in base new; do
      cp abso/${b}_C.so "$SO"
      echo "== $b $rep" >> gpurun_out/attn_ab_$TAG.log
      ITERS=10 timeout -k 10 120 python -u tools/attn_only.py >> gpurun_out/attn_ab_$TAG.log 2>&1
    done
  done
  cp abso/new_C.so "$SO"
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_production.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "attention or dropout or flash or decode" > gpurun_out/attn_tests_$TAG.log 2>&1
  echo "attn tests: $(tail -1 gpurun_out/attn_tests_$TAG.log)"
  grep -A1 "==" gpurun_out/attn_ab_$TAG.log | grep -v "^--" || true
fi
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > gpurun_out/bench_$TAG.log 2>&1
echo "bench: $(tail -1 gpurun_out/bench_$TAG.log | cut -c1-220)"
if [ "${SKIP_EXTRA:-0}" != 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --activation-checkpointing every_layer \
      > gpurun_out/bench_${TAG}_ac.log 2>&1
  echo "ac: $(tail -1 gpurun_out/bench_${TAG}_ac.log | cut -c1-220)"
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --lora > gpurun_out/bench_${TAG}_lora.log 2>&1
  echo "lora: $(tail -1 gpurun_out/bench_${TAG}_lora.log | cut -c1-220)"
fi
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
echo "profile done"
