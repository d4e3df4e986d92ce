# round 5: attention forward issue-priority A/B (SA_FWD_PRIO 1 = softmax VALU at prio 1, 2 = MFMA phases at prio 1)
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in tree prio1 prio2; do
    so=""; [ $v != tree ] && so=$PWD/variants/$v.so
    echo "== $v set $i" >> gpurun_out/r8g_attn.txt
    SCALING_AMD_EXT_SO=$so ITERS=20 timeout -k 10 120 python -u tools/attn_only.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/r8g_attn.txt || exit 1
  done
done
