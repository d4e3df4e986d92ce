#!/bin/bash
# GPU box: graph-decode latency (norm-prologue GEMVs on/off) and a kernel trace whose last 150 ms (inside the graph
# replay of 128 tokens) is summarised per token on the box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-dp}
for i in $(seq 1 ${AB_RUNS:-2}); do
  SCALING_AMD_DECODE_NORM_GEMV=1 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_norm_${i}_$TAG.log 2>&1
  SCALING_AMD_DECODE_NORM_GEMV=0 timeout -k 10 300 python -u tools/decode_bench.py > gpurun_out/dec_nonorm_${i}_$TAG.log 2>&1
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/pd_$TAG -o run -- python3 "$R/tools/decode_bench.py" --tokens 128 \
    > "$R/gpurun_out/dec_prof_$TAG.log" 2>&1
cd "$R"
MS=$(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dec_prof_$TAG.log') if l.startswith('{')][-1]); print(d['graph_ms_per_token'])")
TOK=$(python3 -c "print(int(150 / $MS))")
python tools/rocpd_summary.py /tmp/pd_$TAG/run_results.db --tail-ms 150 --steps $TOK > gpurun_out/dec_kernels_$TAG.md 2>&1 || true
rm -rf /tmp/pd_$TAG
