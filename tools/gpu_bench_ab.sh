#!/bin/bash
# GPU box: 1-GPU 7B bench A/B over an environment switch (ENVVAR=A vs ENVVAR=B, interleaved twice), then
# a rocprofv3 kernel-stats profile with the B setting.  Optional TESTS run first.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
fi
for rep in 1 2; do
  for val in $A $B; do
    env $ENVVAR=$val timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > gpurun_out/bench_${TAG}_${ENVVAR}_${val}_$rep.log 2>&1
    tail -1 gpurun_out/bench_${TAG}_${ENVVAR}_${val}_$rep.log | cut -c1-200
  done
done
if [ "$PROFILE" = "1" ]; then
  export $ENVVAR=$B
  cd /tmp
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 \
      > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
fi
