# round 5: weight-gradient GEMM tile-group height A/B at the 7B shapes (tools/wgrad_bench.py): kGroupM 8 (tree) vs 4
# (variants/wg4.so) vs 16 (variants/wg16.so), interleaved
mkdir -p gpurun_out
for i in 1 2; do
  for v in g8 wg4 wg16; do
    so=""
    [ $v != g8 ] && so=$PWD/variants/$v.so
    echo "$v set $i: $(SCALING_AMD_EXT_SO=$so timeout -k 10 200 python -u tools/wgrad_bench.py 2>&1 | grep TF)" >> gpurun_out/r7h_wgrad.txt || exit 1
  done
done
