# round 5: attention A/B -- XCD-grouped q heads (variants/xcd.so, -DSA_ATTN_XCD=1) vs the default build, interleaved
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base xcd; do
    so=""
    [ $v = xcd ] && so=$PWD/variants/xcd.so
    echo "== $v set $i" >> gpurun_out/r7b_attn.txt
    SCALING_AMD_EXT_SO=$so timeout -k 10 120 python -u tools/attn_only.py >> gpurun_out/r7b_attn.txt 2>&1 || exit 1
  done
done
