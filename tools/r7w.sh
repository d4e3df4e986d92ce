# round 5: NT GEMM round-major remap (tree) vs XCD-contiguous (variants/ntx.so), against hipBLASLt (tools/gemm_nt_bench.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_nt or nt_" > gpurun_out/r7w_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in ntx tree; do
    so=""; [ $v = ntx ] && so=$PWD/variants/ntx.so
    echo "== $v set $i" >> gpurun_out/r7w_nt.txt
    SCALING_AMD_EXT_SO=$so timeout -k 10 400 python -u tools/gemm_nt_bench.py --rounds 2 --iters 8 2>&1 | grep -v amdgpu.ids | grep -v "^{" >> gpurun_out/r7w_nt.txt || exit 1
  done
done
