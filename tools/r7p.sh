# round 5: wgrad GEMM round-major tile remap (tree) vs the XCD-contiguous remap (variants/xcdc.so): GEMM tests,
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
for i in 1 2; do
  for v in xcdc tree; do
    so=""; [ $v = xcdc ] && so=$PWD/variants/xcdc.so
    SCALING_AMD_EXT_SO=$so timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r7p_bench_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(grep '^{' gpurun_out/r7p_bench_${v}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> gpurun_out/r7p_summary.txt
  done
done
