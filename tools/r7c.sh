# round 5: kernel tests on the new build (XCD-grouped attention heads, vectorised AdamW I/O), then bench A/B vs the
# previous build (variants/base.so), interleaved
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r7c_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in base new; do
    so=""
    [ $v = base ] && so=$PWD/variants/base.so
    SCALING_AMD_EXT_SO=$so timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 > gpurun_out/r7c_bench_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(grep '^{' gpurun_out/r7c_bench_${v}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> gpurun_out/r7c_summary.txt
  done
done
