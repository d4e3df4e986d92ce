# round 5: attention on contiguous q / k / v vs views of one packed projection output (the training layout)
mkdir -p gpurun_out
for i in 1 2 3; do
  for pk in 0 1; do
    echo "== packed=$pk set $i" >> gpurun_out/r7t_attn.txt
    PACKED=$pk timeout -k 10 120 python -u tools/attn_only.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/r7t_attn.txt || exit 1
  done
done
