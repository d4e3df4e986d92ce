#!/bin/bash
# GPU box, end of round 3: the 1-GPU headline bench, smoke(), then a graph-phase kernel profile of the decode step.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final_r3.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final_r3.log 2>&1
