# round 5 race forensics: PyTorch's stream sanitizer on the DP2 multi-stream run, and the caching allocator off
mkdir -p gpurun_out
B="--model llama_tiny --backend gloo-gpu --seq-len 256 --micro-batch 2 --steps 3 --warmup 1 --gpus 2"
TORCH_CUDA_SANITIZER=1 SCALING_AMD_DETERMINISTIC=1 timeout -k 10 400 python -u bench.py $B > gpurun_out/r5u_csan.log 2>&1
echo "csan rc=$?" >> gpurun_out/r5u_summary.txt
PYTORCH_NO_CUDA_MEMORY_CACHING=1 SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=5 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5u_trace_nocache.log 2>&1
echo "nocache rc=$?" >> gpurun_out/r5u_summary.txt
SCALING_AMD_SINGLE_STREAM=0 RACE_TRACE_RUNS=5 timeout -k 10 500 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5u_trace_multi.log 2>&1
echo "multi rc=$?" >> gpurun_out/r5u_summary.txt
