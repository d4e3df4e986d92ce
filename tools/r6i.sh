# round 5 final: BASELINE #3 per-rank proxy, TP comm pieces 1 / 2 / 4 interleaved twice (stub collectives: contiguous
# copies), then the SP-gather overlap off
mkdir -p gpurun_out
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r6i_$name.log 2>&1 || exit 1
  grep '^{' gpurun_out/r6i_$name.log | python -c "import sys,json; [print('$name', 'ms', json.loads(l)['ms_per_step'], 'loss', json.loads(l)['config'].get('loss'), 'peak', json.loads(l)['config'].get('peak_mem_gib')) for l in sys.stdin]" >> gpurun_out/r6i_summary.txt
}
P="--shard-proxy baseline3 --steps 5 --warmup 2"
for i in 1 2; do
  run c1_$i X=1 -- $P --tp-comm-chunks 1
  run c2_$i X=1 -- $P --tp-comm-chunks 2
  run c4_$i X=1 -- $P --tp-comm-chunks 4
done
run c4_spov0 SCALING_AMD_SP_OVERLAP=0 -- $P --tp-comm-chunks 4
run c1_spov0 SCALING_AMD_SP_OVERLAP=0 -- $P --tp-comm-chunks 1
