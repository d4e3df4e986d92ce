# round 5: dK/dV segment-major grid (variants/dkseg.so) vs tree (fingerprints + timing), then the 1-GPU bench of the
# tree vs the build before the wgrad round-major remap and the attention segment-major grid (variants/xcdc.so)
mkdir -p gpurun_out
for v in tree dkseg; do
  so=""; [ $v = dkseg ] && so=$PWD/variants/dkseg.so
  SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_bits.py > gpurun_out/r7s_bits_$v.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for v in tree dkseg; do
    so=""; [ $v = dkseg ] && so=$PWD/variants/dkseg.so
    echo "== $v set $i" >> gpurun_out/r7s_attn.txt
    SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_only.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/r7s_attn.txt || exit 1
  done
done
for i in 1 2; do
  for v in xcdc tree; do
    so=""; [ $v = xcdc ] && so=$PWD/variants/xcdc.so
    timeout -k 10 400 env SCALING_AMD_EXT_SO=$so python -u bench.py --steps 10 --warmup 3 > gpurun_out/r7s_bench_${v}_$i.log 2>&1 || exit 1
    echo "$v $i $(grep '^{' gpurun_out/r7s_bench_${v}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> gpurun_out/r7s_summary.txt
  done
done
