#!/bin/bash
# Attention build-variant A/B on one GPU box: numerics tests of every variant .so under variants/, then interleaved
# isolated timings (tools/attn_only.py, 7B step shape) of the tree build and each variant.
#   VARIANTS="nw6 kt128"  (variants/<name>.so, built by SCALING_AMD_FILE_FLAGS=... SCALING_AMD_BUILD_OUT=variants/<name>.so)
#   ROUNDS=2  TESTK="flash or attention"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-ab}
LOG=gpurun_out/attn_ab_$TAG.log
: > "$LOG"
for v in ${VARIANTS}; do
    echo "== tests $v $(date +%T)" >> "$LOG"
    SCALING_AMD_EXT_SO="$R/variants/$v.so" timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q \
        --timeout 120 --timeout-method thread -k "${TESTK:-flash or attention}" >> "$LOG" 2>&1
done
for r in $(seq ${ROUNDS:-2}); do
    echo "== tree round $r $(date +%T)" >> "$LOG"
    timeout -k 10 120 python -u tools/attn_only.py >> "$LOG" 2>&1
    for v in ${VARIANTS}; do
        echo "== $v round $r" >> "$LOG"
        SCALING_AMD_EXT_SO="$R/variants/$v.so" timeout -k 10 120 python -u tools/attn_only.py >> "$LOG" 2>&1
    done
done
echo "== done $(date +%T)" >> "$LOG"
