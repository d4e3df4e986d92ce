# round 5: attention A/B over three builds -- xcd (variants/xcd.so: XCD-grouped heads), skip (variants/skip.so: + fully
# masked wave tiles skipped), fast (tree: + forward fast path without the row max): bit fingerprints (all three must
# agree), kernel tests on the tree build, interleaved timing
mkdir -p gpurun_out
so_of() { case $1 in xcd) echo $PWD/variants/xcd.so ;; skip) echo $PWD/variants/skip.so ;; *) echo "" ;; esac; }
for v in xcd skip fast; do
  SCALING_AMD_EXT_SO=$(so_of $v) timeout -k 10 120 python -u tools/attn_bits.py > gpurun_out/r7f_bits_$v.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or attention or rope" > gpurun_out/r7f_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in xcd skip fast; do
    echo "== $v set $i" >> gpurun_out/r7f_attn.txt
    SCALING_AMD_EXT_SO=$(so_of $v) timeout -k 10 120 python -u tools/attn_only.py >> gpurun_out/r7f_attn.txt 2>&1 || exit 1
  done
done
