#!/bin/bash
# GPU box: 1-GPU 7B bench over micro-batch x grad-acc splits of the same 8-sequence global batch (interleaved).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
for rep in 1 2; do
  for cfg in "2 4" "4 2"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --micro-batch $1 --grad-acc $2 \
        > gpurun_out/bench_${TAG}_mb$1_acc$2_$rep.log 2>&1
    echo "mb$1 acc$2 rep$rep: $(tail -1 gpurun_out/bench_${TAG}_mb$1_acc$2_$rep.log | cut -c1-160)"
  done
done
