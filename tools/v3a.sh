set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "flash_attention" > gpurun_out/v3_tests.log 2>&1
timeout -k 10 120 python -u tools/attn_only.py > gpurun_out/v3_attn.log 2>&1
SCALING_AMD_FA_FWD_V3=0 timeout -k 10 120 python -u tools/attn_only.py > gpurun_out/v2_attn.log 2>&1
bash tools/e1_race.sh
