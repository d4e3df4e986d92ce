#!/bin/bash
# GPU box: optional tests, then the 1-GPU 7B bench A/B over a bench.py flag (FLAG=A vs FLAG=B, interleaved twice).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS ${TESTK:+-k "$TESTK"} -m gpu -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/tests_$TAG.log 2>&1
fi
for rep in 1 2; do
  for val in $A $B; do
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 $FLAG $val > gpurun_out/bench_${TAG}_${val}_$rep.log 2>&1
    echo "$FLAG $val: $(tail -1 gpurun_out/bench_${TAG}_${val}_$rep.log | cut -c1-160)"
  done
done > gpurun_out/bench_ab_$TAG.txt
