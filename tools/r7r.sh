# round 5: wgrad round-major remap microbench (r7p without its bench) + attention segment-major A/B (r7q)
# microbench with hot operands and with 4 rotated operand sets (colder than the MALL), then the 1-GPU bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r7p_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in xcdc tree; do
    so=""; [ $v = xcdc ] && so=$PWD/variants/xcdc.so
    echo "$v hot  $i: $(SCALING_AMD_EXT_SO=$so timeout -k 10 200 python -u tools/wgrad_bench.py 2>&1 | grep TF)" >> gpurun_out/r7p_wgrad.txt || exit 1
    echo "$v cold $i: $(SCALING_AMD_EXT_SO=$so timeout -k 10 300 python -u tools/wgrad_bench.py --cold 4 --iters 8 2>&1 | grep TF)" >> gpurun_out/r7p_wgrad.txt || exit 1
  done
done
bash tools/r7q.sh || exit 1
