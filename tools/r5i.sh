# round 5: attention with / without SLP vectorisation (packed-f32 VALU beside MFMAs), interleaved A/B
set -e
mkdir -p gpurun_out
T="timeout -k 10"
SCALING_AMD_EXT_SO=variants/_C_slpoff.so $T 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash" > gpurun_out/r5i_slpoff_tests.log 2>&1
for rep in 1 2; do
  for v in base slpoff; do
    if [ $v = base ]; then unset SCALING_AMD_EXT_SO; else export SCALING_AMD_EXT_SO=variants/_C_slpoff.so; fi
    echo "== $v rep $rep" >> gpurun_out/r5i_attn_ab.log
    $T 120 python -u tools/attn_only.py >> gpurun_out/r5i_attn_ab.log 2>&1
  done
done
unset SCALING_AMD_EXT_SO
