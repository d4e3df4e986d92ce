#!/bin/bash
# Asynchronous-rehearsal trace of multi-rank runs (CASES="name:bench args;...", default TP2 and TP2 + SP) (SCALING_AMD_REHEARSAL_ASYNC=1, SCALING_AMD_REHEARSAL_TRACE=1): every
# enqueue (Python) and every worker job step (C++) per rank, to find where two ranks' collective orders part.
# A hang ends at the time limit; the per-rank Python stacks are dumped by tools/hang_dump.py into gpurun_out/async_tp/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/async_tp
IFS=";" read -ra CASE_LIST <<< "${CASES:-tp2:--gpus 2 --tp 2;tp2_sp:--gpus 2 --tp 2 --sequence-parallel}"
for case in "${CASE_LIST[@]}"; do
    name=${case%%:*}; args=${case#*:}
    echo "[async_tp] $name $(date +%T)"
    SCALING_AMD_REHEARSAL_ASYNC=1 SCALING_AMD_REHEARSAL_TRACE=1 SCALING_AMD_DETERMINISTIC=1 \
    SCALING_AMD_DEBUG_HOOKS=tools/hang_dump.py HANG_DUMP_S=${HANG_S:-60} \
        timeout -k 10 ${LIMIT:-90} python -u bench.py --model llama_tiny --backend gloo-gpu --seq-len 256 --micro-batch 2 \
        --steps 2 --warmup 0 $args > gpurun_out/async_tp/$name.out 2> gpurun_out/async_tp/$name.err
    echo "[async_tp] $name rc=$?"
    for f in gpurun_out/hang.rank*.txt; do [ -s "$f" ] && mv "$f" "gpurun_out/async_tp/$name.$(basename $f)"; done
done
