#!/bin/bash
# Interleaved A/B of two bench.py argument sets under the driver protocol (20 + 5 steps by default):
#   A="--overlap-step 1" B="--overlap-step 0" ROUNDS=3 TAG=x bash tools/bench_ab.sh
# (ENV_A / ENV_B: extra environment per arm).  One JSON line per run -> gpurun_out/bench_ab_$TAG.jsonl
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-ab}
OUT=gpurun_out/bench_ab_$TAG.jsonl
: > "$OUT"
for r in $(seq ${ROUNDS:-3}); do
    for arm in A B; do
        if [ $arm = A ]; then args=$A; envs=$ENV_A; else args=$B; envs=$ENV_B; fi
        echo "[bench_ab] round $r arm $arm: $args $envs $(date +%T)"
        env $envs timeout -k 10 400 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} $args \
            > gpurun_out/bench_ab_one.log 2>&1 || { tail -20 gpurun_out/bench_ab_one.log; exit 1; }
        grep '^{' gpurun_out/bench_ab_one.log | sed "s/^{/{\"arm\": \"$arm\", \"round\": $r, \"args\": \"$args $envs\", /" >> "$OUT"
    done
done
python - "$OUT" <<'PY'
import json, sys, statistics
rows = [json.loads(l) for l in open(sys.argv[1])]
for arm in "AB":
    ms = [r["ms_per_step"] for r in rows if r["arm"] == arm]
    print(arm, rows[0 if arm == "A" else 1]["args"], "ms/step", [round(m, 1) for m in ms], "median", round(statistics.median(ms), 1))
PY
