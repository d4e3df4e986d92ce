"""Script launched by the runner tests: every rank writes its LaunchConfig as JSON; ``fail_rank`` exits 3
and the other ranks sleep, so the launcher's fail-fast must kill them."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from scaling_amd.core.runner.launch_config import LaunchConfig  # noqa: E402

if __name__ == "__main__":
    config = LaunchConfig.from_launcher_args()
    assert config.payload is not None
    out = Path(config.payload["cache_dir"])
    (out / f"process_{config.global_rank}.json").write_text(config.model_dump_json())
    fail = config.payload.get("fail_rank")
    if fail is not None:
        if config.global_rank == fail:
            sys.exit(3)
        time.sleep(60)
