# round 5: is the TunableOp table applied to the step's forward GEMMs? (table vs heuristic, 3-D vs 2-D F.linear)
mkdir -p gpurun_out
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 240 python -u tools/gemm_table_check.py > gpurun_out/gemm_table_check_r8d.log 2>&1 || exit 1
# which GEMMs of a (2-layer, 7B-width) training step miss the table
cd /tmp && PYTORCH_TUNABLEOP_RECORD_UNTUNED=1 PYTORCH_TUNABLEOP_UNTUNED_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/untuned_r8d.csv \
  timeout -k 10 300 python -u $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --num-layers 2 > $GRAFT_REPO_ROOT/gpurun_out/bench_untuned_r8d.log 2>&1 || exit 1
