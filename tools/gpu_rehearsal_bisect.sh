#!/bin/bash
# GPU box: bisect the multi-rank rehearsal failure over layouts / optimizer switches (Python errors only;
# stops at the first fault-like exit status).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
B="--model llama_tiny --backend gloo-gpu --seq-len 256 --micro-batch 2 --steps 3 --warmup 2"
i=0
while read -r args; do
  i=$((i+1))
  timeout -k 10 120 python -u bench.py $B $args > gpurun_out/bisect_$i.log 2>&1
  rc=$?
  echo "[$rc] $args :: $(grep -o 'grad norm is [a-z/]*\|"dp_param_checksum_agree": [a-z]*' gpurun_out/bisect_$i.log | head -1)"
  case $rc in 0|1) ;; *) echo "stopping at rc=$rc"; exit $rc;; esac
done <<'LIST'
--gpus 2 --grad-acc 2
--gpus 4 --tp 2 --grad-acc 1
--gpus 4 --pp 2 --grad-acc 2
--gpus 4 --pp 2 --grad-acc 2 --lazy-zero 0
--gpus 4 --pp 2 --grad-acc 2 --overlap-step 0
--gpus 4 --pp 2 --grad-acc 2 --zero 0
--gpus 4 --tp 2 --grad-acc 2
--gpus 8 --tp 2 --pp 2 --grad-acc 2 --lazy-zero 0 --overlap-step 0
--gpus 4 --pp 2 --grad-acc 4
--gpus 4 --pp 2 --grad-acc 1
LIST
