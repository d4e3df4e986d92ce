# round 5 race forensics: attention reproducibility beside another process's kernels, many iterations per condition
mkdir -p gpurun_out
for h in none hip_wgrad blas attn; do
  timeout -k 10 260 python -u tools/attn_stress.py --iters 3000 --hammer $h > gpurun_out/r6a_stress_$h.log 2>&1
  rc=$?
  echo "$h rc=$rc $(grep '"hammer"' gpurun_out/r6a_stress_$h.log)" >> gpurun_out/r6a_summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
