#!/bin/bash
# Host-side profile of the BASELINE #2 bench (bench.py --model transformer_example): cProfile of 100 timed steps (SCALING_AMD_BENCH_CPROFILE: the timed loop only)
# (top functions by own and cumulative time) and a kernel trace (launches per step, device busy time).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/example_prof
SCALING_AMD_BENCH_CPROFILE=gpurun_out/example_prof/bench.prof timeout -k 10 300 python -u bench.py \
    --model transformer_example --steps ${STEPS:-100} --warmup 10 > gpurun_out/example_prof/bench.log 2>&1
python - <<'PY' > gpurun_out/example_prof/cprofile_top.txt
import pstats
p = pstats.Stats("gpurun_out/example_prof/bench.prof")
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumtime").print_stats(60)
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/example_prof/prof" -o run -- \
    python3 -u "$R/bench.py" --model transformer_example --steps 20 --warmup 5 > "$R/gpurun_out/example_prof/prof.log" 2>&1
