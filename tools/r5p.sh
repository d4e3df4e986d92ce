# round 5: BASELINE #3 per-rank proxy NaN at 32 layers (2 layers fine): layer-count bisection + path switches
mkdir -p gpurun_out
run() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5p_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o 'grad norm is [a-z/]*' gpurun_out/r5p_$name.log | head -1)" >> gpurun_out/r5p_summary.txt
  grep '^{' gpurun_out/r5p_$name.log | python -c "import sys,json; [print('   loss', json.loads(l)['config'].get('loss'), 'ms', json.loads(l)['ms_per_step']) for l in sys.stdin]" >> gpurun_out/r5p_summary.txt 2>/dev/null
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
P="--shard-proxy baseline3 --steps 1 --warmup 1"
run l8 -- $P --num-layers 8
run l16 -- $P --num-layers 16
run l32 -- $P
run l32_c1_ov0 SCALING_AMD_SP_OVERLAP=0 -- $P --tp-comm-chunks 1
run l32_c1_ov0_ragoff SCALING_AMD_SP_OVERLAP=0 SCALING_AMD_WGRAD_RAGGED=0 SCALING_AMD_DEFER_RESIDUAL=0 -- $P --tp-comm-chunks 1
