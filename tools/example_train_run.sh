#!/bin/bash
# End-to-end run of examples/transformer_example on one MI355X: synthetic corpus, the runner entry point, 50 steps with
# checkpoints at steps 25 and 50 (loss curve in gpurun_out/example_train/train.log).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/example_train
python examples/transformer_example/make_synthetic_data.py examples/transformer_example/data/data \
    > gpurun_out/example_train/data.log 2>&1
rm -rf checkpoints
timeout -k 10 400 python -u -m examples.transformer_example.run examples/transformer_example/config.yml \
    > gpurun_out/example_train/train.log 2>&1
ls -R checkpoints | head -20 > gpurun_out/example_train/checkpoints.txt
