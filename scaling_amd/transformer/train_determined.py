"""Determined-cluster entry (reference ``transformer/train_determined.py``): reads the torch launcher
env, maps Determined hyper-parameters (``target_train_tokens``, ``warmup_tokens``, layout keys) onto
config overrides and runs ``train.main`` with Determined checkpoint/metric reporting.

``determined`` is an optional dependency; without it this module still imports and
``hparams_to_overrides`` is usable, but ``main`` requires a Determined context."""
from __future__ import annotations

import argparse
import os
from typing import Any, Optional

from ..core.runner.launch_config import LaunchConfig
from .context import TransformerConfig
from .train import main as train_main

_TOPOLOGY_KEYS = ("model_parallel_size", "pipe_parallel_size", "sequence_parallel", "global_batch_size",
                  "micro_batch_size", "activation_checkpointing_type", "pipe_partition_method", "pipe_partition_overwrite")


def from_launcher_args_determined(argv: Optional[list[str]] = None) -> LaunchConfig:
    parser = argparse.ArgumentParser(description="process launch")
    parser.add_argument("--config", type=str, default=None, help="path to config file")
    parser.add_argument("remaining_args", nargs=argparse.REMAINDER)
    args = parser.parse_args(argv)
    world = int(os.environ["WORLD_SIZE"])
    payload = None
    if args.config is not None:
        payload = TransformerConfig.from_yaml(args.config, overwrite_values={"topology": {"world_size": world}}).as_dict()
    return LaunchConfig(master_addr=os.environ["MASTER_ADDR"], master_port=os.environ["MASTER_PORT"], world_size=world,
                        global_rank=int(os.environ["RANK"]), local_slot=int(os.environ["LOCAL_RANK"]), payload=payload)


def hparams_to_overrides(hparams: Optional[dict[str, Any]], overwrite_config: Optional[dict[str, Any]] = None
                         ) -> dict[str, Any]:
    """Determined trial hyper-parameters -> nested config overrides (``layout`` sub-dict honoured)."""
    o: dict[str, Any] = dict(overwrite_config or {})
    if hparams and "layout" in hparams:
        hparams = hparams["layout"]
    if not hparams:
        return o
    for k in ("topology", "transformer_architecture", "logger", "trainer", "learning_rate_scheduler"):
        o.setdefault(k, {})
    tokens_per_step = None
    if "global_batch_size" in hparams and "sequence_length" in hparams:
        tokens_per_step = hparams["global_batch_size"] * hparams["sequence_length"]
    if hparams.get("learning_rate"):
        o["learning_rate_scheduler"]["learning_rate"] = hparams["learning_rate"]
    if hparams.get("target_train_tokens"):
        assert tokens_per_step is not None, "target_train_tokens needs global_batch_size and sequence_length"
        o["trainer"]["train_iterations"] = int(hparams["target_train_tokens"] / tokens_per_step)
    if hparams.get("warmup_tokens"):
        assert tokens_per_step is not None, "warmup_tokens needs global_batch_size and sequence_length"
        o["learning_rate_scheduler"]["learning_rate_warmup_steps"] = int(hparams["warmup_tokens"] / tokens_per_step)
    if "wandb_project" in hparams:
        o["logger"]["wandb_project"] = hparams["wandb_project"]
    for k in _TOPOLOGY_KEYS:
        if k in hparams:
            o["topology"][k] = hparams[k]
    if "train_iterations" in hparams:
        o["trainer"]["train_iterations"] = hparams["train_iterations"]
    if "kernel" in hparams:
        o["transformer_architecture"]["masked_softmax"] = {"kernel": hparams["kernel"]}
    if "sequence_length" in hparams:
        o["transformer_architecture"]["sequence_length"] = hparams["sequence_length"]
    return o


def main(determined_context: Any, profiler: Any, overwrite_config: Optional[dict] = None, return_metrics: bool = False,
         det_experiment_id: Optional[int] = None, det_trial_id: Optional[int] = None, info: Any = None
         ) -> Optional[list[dict[str, Any]]]:
    launch_config = from_launcher_args_determined([])
    o = dict(overwrite_config or {})
    o.setdefault("runner", {})["use_determined"] = True
    o["determined_experiment_id"] = det_experiment_id
    o["determined_trial_id"] = det_trial_id
    o = hparams_to_overrides(info.trial.hparams if info is not None else None, o)
    return train_main(launch_config, overwrite_config=o, return_metrics=return_metrics,
                      determined_context=determined_context, determined_profiler=profiler)


if __name__ == "__main__":  # pragma: no cover - requires a Determined cluster
    from ..core.determined import init as det_init  # type: ignore[attr-defined]

    with det_init() as ctx:
        main(ctx, None)
