# round 5: SwiGLU kernels with two 16-B chunks per thread and 32-bit chunk indexing (tree) vs before (variants/prev.so)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "swiglu" > gpurun_out/r7j_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in prev tree; do
    so=""; [ $v = prev ] && so=$PWD/variants/prev.so
    echo "== $v set $i" >> gpurun_out/r7j_swiglu.txt
    SCALING_AMD_EXT_SO=$so timeout -k 10 200 python -u tools/swiglu_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/r7j_swiglu.txt || exit 1
  done
done
