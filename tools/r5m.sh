# round 5: chunked SP proxy test (after the strided-matmul fault fix), DP2 race traces, BASELINE #3/#4 proxies
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -x -v --timeout 250 --timeout-method thread -k "shard_proxy" > gpurun_out/r5m_proxy_test.log 2>&1
bash tools/r5l.sh
