# round 5 race forensics: kernel timeline of the DP2 multi-stream rehearsal (both ranks), to list what runs beside the
# attention backward in the same process
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6c_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model llama_tiny --backend gloo-gpu --seq-len 256 --micro-batch 2 --steps 3 --warmup 1 --gpus 2 > $GRAFT_REPO_ROOT/gpurun_out/r6c_prof.log 2>&1
