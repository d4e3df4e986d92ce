# round 5: attention grid order -- segment-major (tree: q tiles of few segments resident together) vs tile-major
# (variants/seg0.so); bit fingerprints must agree; attention tests; isolated timing interleaved
mkdir -p gpurun_out
for v in seg0 tree; do
  so=""; [ $v = seg0 ] && so=$PWD/variants/seg0.so
  SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_bits.py > gpurun_out/r7q_bits_$v.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or attention or rope" > gpurun_out/r7q_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in seg0 tree; do
    so=""; [ $v = seg0 ] && so=$PWD/variants/seg0.so
    echo "== $v set $i" >> gpurun_out/r7q_attn.txt
    SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_only.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/r7q_attn.txt || exit 1
  done
done
