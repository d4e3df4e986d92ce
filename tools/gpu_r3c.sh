#!/bin/bash
# GPU box: full GPU test suite + smoke, then the wgrad layout probe with TunableOp-tuned hipBLASLt layouts.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r3c}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 400 python -u tools/gemm_layout_probe.py --tune > gpurun_out/gemm_layout_probe_tuned_$TAG.log 2>&1
