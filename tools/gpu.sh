#!/bin/bash
# One entry point for GPU-box runs (gpurun -- 'bash tools/gpu.sh STEP ...'): every step runs under its own time limit,
# writes gpurun_out/<step>_<TAG>.log, and the script stops at the first failing step (set -e), so a fault or a hang
# never starts another GPU step in the same call.
#   tests      pytest -m gpu (whole GPU suite; PYTEST_K narrows it)
#   smoke      __graft_entry__.smoke()
#   bench      1-GPU bench.py (BENCH_ARGS)
#   prof       rocprofv3 --kernel-trace --stats of 3 bench steps + per-category summary of the last step
#   pmc        SQ/MFMA counters of every kernel of a 4-layer 7B-width step (PMC_PROG / PMC_ARGS: another program)
#   attn       tools/attn_only.py (isolated attention at the 7B shape)
#   decode     tools/decode_bench.py
#   race       the multi- vs single-stream race check (tests/test_gpu_rehearsal.py -k race_check)
#   race_bisect  tools/race_bisect.py: which side stream makes a layout differ from its single-stream twin
#   race_trace   tools/race_trace.py: the first step / quantity where two identical runs differ
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-run}
T="timeout -k 10"
PY="python -u"
for step in "$@"; do
    echo "[gpu.sh] $step $(date +%T)"
    case "$step" in
    tests)
        $T 1000 $PY -m pytest tests -m gpu -v --durations=40 --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
            > gpurun_out/tests_$TAG.log 2>&1 ;;
    smoke)
        $T 180 $PY -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 ;;
    bench)
        $T 600 $PY bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench_$TAG.log 2>&1 ;;
    prof)
        (cd /tmp && export TMPDIR=/tmp && $T 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run \
            -- python3 "$R/bench.py" ${PROF_ARGS:---steps 3 --warmup 1} > "$R/gpurun_out/prof_$TAG.log" 2>&1)
        $PY tools/rocpd_step.py gpurun_out/prof_$TAG/run_results.db > gpurun_out/prof_step_$TAG.md 2>&1 || true ;;
    pmc)
        B="${PMC_PROG:-$R/bench.py} ${PMC_ARGS:---steps 1 --warmup 1 --num-layers 4}"
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
            SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
            GRBM_GUI_ACTIVE GRBM_COUNT -d "$R/gpurun_out/pmc_$TAG" -o a --output-format csv -- python3 $B \
            > "$R/gpurun_out/pmc_$TAG.log" 2>&1)
        $PY tools/pmc_csv_summary.py gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.txt 2>&1 || true ;;
    attn)
        $T 300 $PY tools/attn_only.py ${ATTN_ARGS:-} > gpurun_out/attn_$TAG.log 2>&1 ;;
    decode)
        $T 300 $PY tools/decode_bench.py ${DECODE_ARGS:-} > gpurun_out/decode_$TAG.log 2>&1 ;;
    race)
        $T 600 $PY -m pytest tests/test_gpu_rehearsal.py -m gpu -x -v --timeout 300 --timeout-method thread \
            -k "race_check" > gpurun_out/race_$TAG.log 2>&1 ;;
    race_bisect)
        $T 900 $PY tools/race_bisect.py ${RACE_ARGS:-} > gpurun_out/race_bisect_$TAG.log 2>&1 ;;
    race_trace)
        $T 600 $PY tools/race_trace.py ${RACE_ARGS:-} > gpurun_out/race_trace_$TAG.log 2>&1 ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
echo "[gpu.sh] done $(date +%T)"
