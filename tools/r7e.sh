# round 5: attention forward fast path (no row max while the tile row sum stays <= 128): bit fingerprint vs the
# previous build (variants/skip.so), kernel tests, then interleaved timing
mkdir -p gpurun_out
for v in skip fast; do
  so=""
  [ $v = skip ] && so=$PWD/variants/skip.so
  SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_bits.py > gpurun_out/r7e_bits_$v.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or attention or rope" > gpurun_out/r7e_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in skip fast; do
    so=""
    [ $v = skip ] && so=$PWD/variants/skip.so
    echo "== $v set $i" >> gpurun_out/r7e_attn.txt
    SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_only.py >> gpurun_out/r7e_attn.txt 2>&1 || exit 1
  done
done
