# round 5: in-step A/B of the SwiGLU backward on the NT dgrad epilogue (7B bench, interleaved), then race sanitizers
mkdir -p gpurun_out
for rep in 1 2; do
  for m in 0 auto; do
    echo "== SCALING_AMD_SWIGLU_BWD_NT=$m rep $rep" >> gpurun_out/r5v_swiglu_ab.log
    SCALING_AMD_SWIGLU_BWD_NT=$m timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 2>&1 | grep '^{' >> gpurun_out/r5v_swiglu_ab.log || exit 1
  done
done
bash tools/r5u.sh
