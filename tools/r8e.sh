# round 5: re-tune the step's hipBLASLt shapes with the chip already at its sustained clock, then A/B the table
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 60 python -u tools/gemm_sustained.py --shape gate_up --seconds 5 --idle-first 0 > gpurun_out/preheat_r8e.log 2>&1 || exit 1
SCALING_AMD_GEMM_RETUNE=1 SCALING_AMD_GEMM_TUNE_ITERS=${ITERS:-20} timeout -k 10 480 python -u bench.py --gemm-tuning tune \
  --gemm-tuning-out $R/gpurun_out/gemm_hot_r8e.csv --steps 1 --warmup 0 > gpurun_out/tune_r8e.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python -u bench.py --steps 10 --warmup 3 2>&1 | grep '^{' | sed "s/^/old $i /" >> gpurun_out/ab_r8e.log || exit 1
  SCALING_AMD_GEMM_TABLE=$R/gpurun_out/gemm_hot_r8e.csv timeout -k 10 150 python -u bench.py --steps 10 --warmup 3 2>&1 | grep '^{' | sed "s/^/hot $i /" >> gpurun_out/ab_r8e.log || exit 1
done
