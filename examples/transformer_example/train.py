"""Per-process entry for the transformer example (runner -> launcher -> this script)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from scaling_amd.core.runner.launch_config import LaunchConfig  # noqa: E402
from scaling_amd.transformer.train import main  # noqa: E402

if __name__ == "__main__":
    main(LaunchConfig.from_launcher_args())
