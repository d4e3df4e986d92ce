"""Entry point for end-to-end training tests: `python -m torch.distributed.run ... tests/train_helper.py <json>`.
Rank 0 writes the per-step metrics to <out>."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from scaling_amd.core.runner.launch_config import LaunchConfig  # noqa: E402
from scaling_amd.transformer.train import main  # noqa: E402

if __name__ == "__main__":
    spec = json.loads(open(sys.argv[1]).read())
    metrics = main(LaunchConfig.from_launcher_args([]), overwrite_config=spec["config"], return_metrics=True)
    if int(os.environ.get("RANK", "0")) == 0:
        with open(spec["out"], "w") as f:
            json.dump(metrics, f)
