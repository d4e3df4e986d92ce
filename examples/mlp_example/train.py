"""Per-process MLP training entry (started by run.py through the runner / launcher, or torchrun)."""
from __future__ import annotations

import os
import sys
from pathlib import Path
from typing import Any, Optional

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from scaling_amd.core import BaseTrainer, Topology  # noqa: E402
from scaling_amd.core.topology import shutdown_distributed  # noqa: E402
from scaling_amd.core.logging import logger  # noqa: E402
from scaling_amd.core.runner import LaunchConfig  # noqa: E402

from examples.mlp_example.config import MLPConfig  # noqa: E402
from examples.mlp_example.context import MLPContext  # noqa: E402
from examples.mlp_example.data import MNISTDataset  # noqa: E402
from examples.mlp_example.model import init_model, init_optimizer, loss_function, metrics_aggregation_fn  # noqa: E402


def main(launch_config: LaunchConfig, overwrite_config: Optional[dict] = None, return_metrics: bool = False
         ) -> Optional[list[dict[str, Any]]]:
    d = launch_config.overwrite_config_dict_with_launcher_args(dict(launch_config.payload or overwrite_config or {}))
    config = MLPConfig.from_dict(d)
    topology = Topology(config=config.topology)
    context = MLPContext(config=config, topology=topology)
    logger.configure(config=config.logger, name=f"RANK {topology.config.global_rank}", global_rank=topology.config.global_rank)
    context.initialize(master_addr=launch_config.master_addr, master_port=str(launch_config.master_port),
                       seed=config.trainer.seed)
    model = init_model(context=context)
    optimizer = init_optimizer(context=context, model=model)
    train_data = valid_data = None
    if topology.is_io_rank:
        root = Path(config.data.mnist_root)
        train_data = MNISTDataset(root, train=True, synthetic_samples=config.data.synthetic_samples)
        valid_data = MNISTDataset(root, train=False, synthetic_samples=config.data.synthetic_samples)
    trainer = BaseTrainer(config=context.config.trainer, context=context, parallel_module=model, optimizer=optimizer,
                          dataset=train_data, dataset_evaluation=valid_data,
                          sync_batch_to_model_parallel=MNISTDataset.sync_batch_to_model_parallel,
                          metrics_aggregation_fn=metrics_aggregation_fn, loss_function=loss_function)
    metrics = trainer.run_training(return_metrics=return_metrics)
    shutdown_distributed()
    return metrics


if __name__ == "__main__":
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    main(LaunchConfig.from_launcher_args())
