#!/bin/bash
# GPU box (1 GPU): rehearse the multi-rank RCCL paths with several ranks sharing the one card.
# Step 1 checks that RCCL accepts two ranks on one device; only then the DP / TP / PP bench layouts
# run on a 2-layer 7B-width model (debug size, not the headline number).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 90 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29701 tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1
for L in "--tp 1 --pp 1" "--tp 2 --pp 1" "--tp 1 --pp 2" "--tp 2 --pp 1 --sequence-parallel"; do
  timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29702 bench.py --gpus 2 --steps 3 --warmup 1 --num-layers 2 --share-gpu $L \
      >> gpurun_out/rehearsal_2rank.log 2>&1
done
