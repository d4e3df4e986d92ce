# round 5 race forensics: fused attention reproducibility beside a whole llama_tiny training process
mkdir -p gpurun_out
timeout -k 10 280 python -u tools/attn_stress.py --iters 20000 --hammer bench > gpurun_out/r6e_stress_bench.log 2>&1
echo "bench rc=$? $(grep '"hammer"' gpurun_out/r6e_stress_bench.log)" >> gpurun_out/r6e_summary.txt
