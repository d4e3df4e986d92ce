# round 5: attention backward with dQ on a side stream beside dK/dV (default) vs one stream (SCALING_AMD_FA_BWD_STREAMS=0)
mkdir -p gpurun_out
for m in 0 1; do
  SCALING_AMD_FA_BWD_STREAMS=$m timeout -k 10 120 python -u tools/attn_bits.py > gpurun_out/r7o_bits_$m.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or attention or rope" > gpurun_out/r7o_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for m in 0 1; do
    echo "== streams=$m set $i" >> gpurun_out/r7o_attn.txt
    SCALING_AMD_FA_BWD_STREAMS=$m timeout -k 10 120 python -u tools/attn_only.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/r7o_attn.txt || exit 1
  done
done
for i in 1 2; do
  for m in 0 1; do
    SCALING_AMD_FA_BWD_STREAMS=$m timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r7o_bench_${m}_$i.log 2>&1 || exit 1
    echo "streams=$m $i $(grep '^{' gpurun_out/r7o_bench_${m}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> gpurun_out/r7o_summary.txt
  done
done
