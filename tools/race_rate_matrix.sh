#!/bin/bash
# The race-rate probe (tools/race_rate.sh, tree build) under the switches that r5 saw remove the divergence: caching
# allocator off, each side stream folded, all folded, device syncs around the attention backward; plus one rank alone.
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
T=${TAG:-m}
TAG=${T}_base bash tools/race_rate.sh
TAG=${T}_noalloc EXTRA_ENV="PYTORCH_NO_CUDA_MEMORY_CACHING=1" bash tools/race_rate.sh
TAG=${T}_fold_dp EXTRA_ENV="SCALING_AMD_SINGLE_STREAM=dp_comm" bash tools/race_rate.sh
TAG=${T}_fold_opt EXTRA_ENV="SCALING_AMD_SINGLE_STREAM=opt_step" bash tools/race_rate.sh
TAG=${T}_fold_all EXTRA_ENV="SCALING_AMD_SINGLE_STREAM=1" bash tools/race_rate.sh
TAG=${T}_sync EXTRA_ENV="ATTN_FORENSICS_SYNC=1" bash tools/race_rate.sh
TAG=${T}_one GPUS=1 bash tools/race_rate.sh
