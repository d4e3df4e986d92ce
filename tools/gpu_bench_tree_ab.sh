#!/bin/bash
# GPU box: 1-GPU bench A/B between the current tree and an older tree in ./abtree (same native build), interleaved.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for rep in 1 2; do
  (cd abtree && timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > "$R/gpurun_out/ab_old_$rep.log" 2>&1)
  echo "old $rep: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$rep.log)"
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/ab_new_$rep.log 2>&1
  echo "new $rep: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$rep.log)"
done
