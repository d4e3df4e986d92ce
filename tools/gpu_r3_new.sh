#!/bin/bash
# GPU box: the round-3 additions (one-shot all-reduce timeout, small-linear autograd, fp32 flash refusal,
# fp16 loss-scaling rehearsal, deterministic-torch training, delayed-comm race check), then the wgrad layout probe.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r3}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_custom_allreduce.py \
    "tests/test_kernels_gpu.py::test_flash_attention_rejects_fp32" \
    "tests/test_kernels_gpu.py::test_small_linear_keeps_autograd" \
    "tests/test_gpu_rehearsal.py::test_rehearsal_fp16_loss_scaling_resume_bit_exact_gpu" \
    "tests/test_gpu_rehearsal.py::test_deterministic_torch_training_gpu" \
    "tests/test_gpu_rehearsal.py::test_race_check_multi_stream_equals_single_stream" \
    > gpurun_out/new_tests_$TAG.log 2>&1
timeout -k 10 250 python -u tools/gemm_layout_probe.py > gpurun_out/gemm_layout_probe.log 2>&1
