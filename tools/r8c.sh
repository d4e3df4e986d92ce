# round 5: sustained-load rate of the step's hipBLASLt shapes (is the in-step vs tuning-table gap the held clock?)
mkdir -p gpurun_out
for s in gate_up down qkv; do
  timeout -k 10 120 python -u tools/gemm_sustained.py --shape $s --seconds 4 >> gpurun_out/gemm_sustained_r8c.log 2>&1 || exit 1
done
