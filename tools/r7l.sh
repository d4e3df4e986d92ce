# round 5 timing probes (results wrong by design): attention with LDS-DMA loads out of range (probe1), without the
# loop's workgroup barrier (probe2), both (probe3), vs the tree build
mkdir -p gpurun_out
for i in 1 2; do
  for v in tree probe1 probe4; do
    so=""; [ $v != tree ] && so=$PWD/variants/$v.so
    echo "== $v set $i" >> gpurun_out/r7m_probe.txt
    SCALING_AMD_EXT_SO=$so ITERS=5 timeout -k 10 120 python -u tools/attn_only.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/r7m_probe.txt || exit 1
  done
done
