#!/bin/bash
# GPU box: ring wgrad GEMM as the default: gemm tests + determinism stress, production-shape GPU tests, 7B bench
# (ring default vs variant 2 A/B in one session), kernel profile of the step.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r3f}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_tn" -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tests_gemm_$TAG.log 2>&1
for V in 10 13; do timeout -k 10 300 python -u tools/gemm_repeat_check.py $V 20 >> gpurun_out/repeat_$TAG.log 2>&1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/tests_prod_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1
SCALING_AMD_GEMM_VARIANT=2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_v2_$TAG.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 \
    > "$R/gpurun_out/bench_prof_$TAG.log" 2>&1
cd "$R"
python tools/rocpd_step.py /tmp/prof_$TAG/run_results.db > gpurun_out/step_$TAG.md 2>&1 || true
rm -rf /tmp/prof_$TAG
