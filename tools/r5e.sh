# per-rank proxy (collectives stubbed): compute cost of the chunked TP path (BASELINE #3 layout) at 1 / 2 / 4 pieces
set -e
mkdir -p gpurun_out
for c in 1 2 4; do
  timeout -k 10 400 python -u bench.py --shard-proxy baseline3 --tp-comm-chunks $c --steps 4 --warmup 2 > gpurun_out/r5e_proxy3_chunks$c.log 2>&1
done
