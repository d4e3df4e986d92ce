#!/bin/bash
# Per-rank proxies of BASELINE #3 / #4 on one GPU (bench.py --shard-proxy), stub vs emulated collectives
# (--proxy-comm emulate: modelled xGMI time + HBM traffic on 16 CUs per collective), TP comm chunks 1/2/4 and the
# BASELINE #4 micro-batching (4 x 4, 2 x 8, 1 x 16); ONLY=baseline4 skips the baseline3 rows.  One JSON line per run -> gpurun_out/proxy_$TAG.jsonl.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r6}
OUT=gpurun_out/proxy_$TAG.jsonl
: > "$OUT"
run() {
    echo "[proxy] $* $(date +%T)"
    timeout -k 10 400 python -u bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} "$@" > gpurun_out/proxy_one.log 2>&1 || {
        tail -20 gpurun_out/proxy_one.log; exit 1; }
    grep '^{' gpurun_out/proxy_one.log | sed "s/^{/{\"args\": \"$*\", /" >> "$OUT"
}
if [ "${ONLY:-}" != baseline4 ]; then
    for mode in stub emulate; do
        for c in 1 2 4; do
            run --shard-proxy baseline3 --proxy-comm $mode --tp-comm-chunks $c
        done
    done
fi
for mb in "4 4" "2 8" "1 16"; do
    set -- $mb
    run --shard-proxy baseline4 --proxy-comm emulate --micro-batch $1 --grad-acc $2
done
run --shard-proxy baseline4 --proxy-comm stub
run --shard-proxy baseline4_save_matmuls --proxy-comm emulate
echo "[proxy] done $(date +%T)"
