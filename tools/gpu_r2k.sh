#!/bin/bash
# GPU box: GPU test suite + smoke (lazy gradient zeroing, dK/dV loop cursors), interleaved bench A/B of
# --lazy-zero 0/1, then the same-hardware reference baseline: the unmodified reference (scratch copy shipped as
# refsrc.tar.gz, not part of the repository) training the 7B shape on this GPU (tools/reference_bench/).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r2k}
( while true; do sleep 50; echo "tick $(date +%T)"; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null || true' EXIT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo "tests: $(tail -1 gpurun_out/gpu_tests_$TAG.log)"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  echo "smoke ok"
fi
for rep in 1 2; do
  for lz in 0 1; do
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --lazy-zero $lz > gpurun_out/bench_${TAG}_lz${lz}_$rep.log 2>&1
    echo "lazy-zero $lz rep$rep: $(tail -1 gpurun_out/bench_${TAG}_lz${lz}_$rep.log | cut -c1-230)"
  done
done
if [ -f refsrc.tar.gz ]; then
  mkdir -p /tmp/refsrc && tar xzf refsrc.tar.gz -C /tmp/refsrc
  for cfg in "1 8" "2 4"; do
    set -- $cfg
    timeout -k 10 600 python -u tools/reference_bench/ref_bench.py --ref-src /tmp/refsrc/src --steps 3 --warmup 1 \
        --micro-batch $1 --grad-acc $2 > gpurun_out/ref_bench_${TAG}_mb$1.log 2>&1
    echo "reference mb$1: $(tail -1 gpurun_out/ref_bench_${TAG}_mb$1.log | cut -c1-300)"
  done
fi
