# round 5: per-shape wgrad tile-group height (tree: 4 for tall outputs, else 8) vs fixed 8 (variants/g8.so): GEMM tests,
# wgrad microbench, then 1-GPU bench interleaved
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r7i_tests.log 2>&1 || exit 1
for v in tree g8; do
  so=""; [ $v = g8 ] && so=$PWD/variants/g8.so
  echo "$v: $(SCALING_AMD_EXT_SO=$so timeout -k 10 200 python -u tools/wgrad_bench.py 2>&1 | grep TF)" >> gpurun_out/r7i_wgrad.txt || exit 1
done
for i in 1 2; do
  for v in g8 tree; do
    so=""; [ $v = g8 ] && so=$PWD/variants/g8.so
    SCALING_AMD_EXT_SO=$so timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r7i_bench_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(grep '^{' gpurun_out/r7i_bench_${v}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> gpurun_out/r7i_summary.txt
  done
done
