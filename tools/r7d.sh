# round 5: attention with fully-masked wave tiles skipped (new build) vs the XCD build without the skip
# (variants/xcd.so), interleaved; then the attention kernel tests on the new build
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or attention or rope" > gpurun_out/r7d_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in xcd skip; do
    so=""
    [ $v = xcd ] && so=$PWD/variants/xcd.so
    echo "== $v set $i" >> gpurun_out/r7d_attn.txt
    SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_only.py >> gpurun_out/r7d_attn.txt 2>&1 || exit 1
  done
done
