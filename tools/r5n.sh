# round 5: where does the BASELINE #3 per-rank proxy go NaN (7B shard shapes, 2 layers)?  + race fold bisection
mkdir -p gpurun_out
run() {  # name, env..., -- args ; a Python failure (rc 1) moves on, a fault / abort / timeout ends the script
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5n_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/r5n_summary.txt
  grep '^{' gpurun_out/r5n_$name.log | python -c "import sys,json; [print('   loss', json.loads(l)['config'].get('loss'), 'ms', json.loads(l)['ms_per_step']) for l in sys.stdin]" >> gpurun_out/r5n_summary.txt 2>/dev/null
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
P="--shard-proxy baseline3 --num-layers 2 --steps 2 --warmup 1"
run p3_c1_ov1 SCALING_AMD_SP_OVERLAP=1 -- $P --tp-comm-chunks 1
run p3_c4_ov1 SCALING_AMD_SP_OVERLAP=1 -- $P --tp-comm-chunks 4
run p3_c1_ov0 SCALING_AMD_SP_OVERLAP=0 -- $P --tp-comm-chunks 1
run p3_c1_ov0_ragoff SCALING_AMD_SP_OVERLAP=0 SCALING_AMD_WGRAD_RAGGED=0 -- $P --tp-comm-chunks 1
run p3_c1_ov0_mb1 SCALING_AMD_SP_OVERLAP=0 -- $P --tp-comm-chunks 1 --micro-batch 1
for f in dp_comm opt_step; do
  SCALING_AMD_SINGLE_STREAM=$f RACE_TRACE_RUNS=3 timeout -k 10 400 python -u tools/race_trace.py --gpus 2 > gpurun_out/r5n_trace_fold_$f.log 2>&1 || exit $?
done
