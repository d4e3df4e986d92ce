#!/bin/bash
# Rate of attention backwards that differ from a recomputation in place (tools/attn_forensics.py) in the 2-rank
# rehearsal (two processes' waves on the same CUs), per extension build: the tree's and each VARIANTS=<name>
# (variants/<name>.so).  -> gpurun_out/race_rate_$TAG/<build>.rank<r>.json
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${TAG:-r6}
D=gpurun_out/race_rate_$TAG
mkdir -p "$D"
for b in tree ${VARIANTS}; do
    so=""
    [ "$b" != tree ] && so="$R/variants/$b.so"
    echo "[race_rate] $b $(date +%T)"
    SCALING_AMD_EXT_SO=$so SCALING_AMD_DEBUG_HOOKS=tools/attn_forensics.py ATTN_FORENSICS_TWICE=1 \
        ATTN_FORENSICS_OUT="$D/$b" SCALING_AMD_DETERMINISTIC=1 env ${EXTRA_ENV} \
        timeout -k 10 ${RATE_TIMEOUT:-300} python -u bench.py --model llama_tiny --backend gloo-gpu --gpus ${GPUS:-2} --seq-len 256 \
        --micro-batch 2 --steps ${STEPS:-200} --warmup 2 > "$D/$b.log" 2>&1
    cat "$D/$b".rank*.json; echo
done
