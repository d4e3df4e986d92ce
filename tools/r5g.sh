# round-5: attention loop barriers retire every wave's LDS-DMA (dma_barrier): kernel tests, timing, race check w/o xfail
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "flash or gemm_tn" > gpurun_out/r5g_kernel_tests.log 2>&1
$T 120 python -u tools/attn_only.py > gpurun_out/r5g_attn.log 2>&1
CAUSAL=0 $T 120 python -u tools/attn_only.py > gpurun_out/r5g_attn_noncausal.log 2>&1
SCALING_AMD_FA_FWD_V3=1 CAUSAL=0 $T 120 python -u tools/attn_only.py > gpurun_out/r5g_attn_v3_noncausal.log 2>&1
$T 900 python -u -m pytest tests/test_gpu_rehearsal.py -x -v --timeout 400 --timeout-method thread -k "race_check" > gpurun_out/r5g_race.log 2>&1
bash tools/r5d.sh
bash tools/r5e.sh
