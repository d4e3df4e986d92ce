"""Training loop, checkpoint policy and metric logging (reference ``core/trainer/trainer.py:33-558``).

Same checkpoint directory layout (``save_dir/global_step{N}/`` + ``latest``), same resume semantics
(model -> optimizer or refresh -> context), same metric names.  ``DeterminedBaseTrainer`` keeps the
API; the Determined cluster integration is import-guarded (determined is not in the MI355X image).
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Callable, Generic, Optional, TypeVar

import torch

from ..utils.watchdog import HangWatchdog
from ..context import BaseContext, DeterminedBaseContext
from ..data import BaseDataset, DataLoader
from ..logging import logger
from ..nn import ParallelModule, ParallelSelfAttention
from ..optimizer import BaseOptimizer
from .trainer_config import TrainerConfig

BaseContextGeneric = TypeVar("BaseContextGeneric", bound=BaseContext)
ParallelModuleGeneric = TypeVar("ParallelModuleGeneric", bound=ParallelModule)


class BaseTrainer(Generic[BaseContextGeneric, ParallelModuleGeneric]):
    def __init__(
        self,
        config: TrainerConfig,
        context: BaseContextGeneric,
        parallel_module: ParallelModuleGeneric,
        optimizer: BaseOptimizer,
        dataset: Optional[BaseDataset],
        sync_batch_to_model_parallel: Callable,
        loss_function: Callable,
        metrics_aggregation_fn: Optional[Callable] = None,
        dataset_evaluation: Optional[BaseDataset] = None,
    ):
        self.config = config
        self.context = context
        self.parallel_module = parallel_module
        self.parameters_total, self.parameters_unique = parallel_module.get_params_count()
        logger.log_config_dict({"parameters_total": self.parameters_total, "parameters_unique": self.parameters_unique})
        logger.info(f"parameters total {self.parameters_total} unique {self.parameters_unique}")
        self.optimizer = optimizer
        self.dataset = dataset
        self.dataset_evaluation = dataset_evaluation
        loaded = self.load_checkpoint(
            load_dir=config.load_dir,
            load_optimizer_states=config.load_optimizer_states,
            load_context=config.load_context,
            allowed_missing_keys_in_checkpoint=config.allowed_missing_keys_in_checkpoint,
            allowed_unexpected_keys_in_checkpoint=config.allowed_unexpected_keys_in_checkpoint,
            ignore_keys_in_checkpoint=config.ignore_keys_in_checkpoint,
        )
        if config.assert_checkpoint_loaded:
            assert loaded, (
                "checkpoint could not be loaded. if this is intended you may change the parameter "
                "'assert_checkpoint_loaded' in the TrainerConfig to False."
            )
        if config.merge_lora_after_loading_checkpoint:
            for m in parallel_module.modules():
                if isinstance(m, ParallelSelfAttention) and getattr(m, "lora_config", None):
                    m.merge_lora_weights()
            self.optimizer.refresh_optimizer_after_model_change()
            logger.info("Merged LoRa weights")
        self.dataloader: Optional[DataLoader] = None
        self.dataloader_evaluation: Optional[DataLoader] = None
        if context.topology.is_io_rank:
            assert dataset is not None
            kw = dict(topology=context.topology, num_workers=config.dataloader_num_workers,
                      pin_memory=config.dataloader_pin_memory, prefetch_factor=config.dataloader_prefetch_factor)
            self.dataloader = DataLoader(seed=config.seed, consumed_samples=context.consumed_samples, dataset=dataset, **kw)
            if dataset_evaluation is not None:
                self.dataloader_evaluation = DataLoader(seed=config.seed,
                                                        consumed_samples=context.consumed_samples_evaluation,
                                                        dataset=dataset_evaluation, **kw)
        self.sync_batch_to_model_parallel = sync_batch_to_model_parallel
        self.loss_function = loss_function
        self.metrics_aggregation_fn = metrics_aggregation_fn

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoint(self, save_dir: Optional[Path] = None) -> Path:
        save_dir = Path(save_dir or self.config.save_dir)  # type: ignore[arg-type]
        it_dir = save_dir / f"global_step{self.context.iterations}"
        it_dir.mkdir(exist_ok=True, parents=True)
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        self.parallel_module.save_checkpoint(it_dir, separate_file_for_parameters=self.config.separate_file_for_parameters)
        self.optimizer.save_checkpoint(it_dir)
        self.context.save_checkpoint(it_dir)
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        if self.context.topology.config.global_rank == 0:
            with open(save_dir / "latest", "w", encoding="UTF-8") as f:
                f.write(f"global_step{self.context.iterations}")
        logger.info(f"saved checkpoint: {it_dir}")
        return save_dir

    def load_checkpoint(
        self,
        load_dir: Optional[Path] = None,
        load_optimizer_states: bool = True,
        load_context: bool = True,
        allowed_missing_keys_in_checkpoint: Optional[list[str]] = None,
        allowed_unexpected_keys_in_checkpoint: Optional[list[str]] = None,
        ignore_keys_in_checkpoint: Optional[list[str]] = None,
    ) -> bool:
        if load_dir is None:
            return False
        load_dir = Path(load_dir)
        if (load_dir / "latest").is_file():
            it_dir = load_dir / (load_dir / "latest").read_text(encoding="UTF-8").strip()
        elif any(load_dir.glob("*.pt")):
            logger.info(f"no latest file found, using load dir directly instead: {load_dir}")
            it_dir = load_dir
        else:
            logger.error(f"no files found in load dir: {load_dir}")
            return False
        if not it_dir.is_dir():
            logger.error(f"iteration_dir does not exist: {it_dir}")
            return False
        self.parallel_module.load_checkpoint(
            it_dir,
            allowed_missing_keys_in_checkpoint=allowed_missing_keys_in_checkpoint,
            allowed_unexpected_keys_in_checkpoint=allowed_unexpected_keys_in_checkpoint,
            ignore_keys_in_checkpoint=ignore_keys_in_checkpoint,
        )
        if load_optimizer_states:
            self.optimizer.load_checkpoint(it_dir)
        else:
            self.optimizer.refresh_optimizer_after_model_change()
        if load_context:
            self.context.load_checkpoint(it_dir)
        logger.info(f"loaded checkpoint: {it_dir}")
        return True

    # ------------------------------------------------------------------ steps
    def train_step(self) -> Any:
        out = self.parallel_module.train_step(
            dataloader=self.dataloader, optimizer=self.optimizer,
            sync_batch_to_model_parallel=self.sync_batch_to_model_parallel, loss_function=self.loss_function,
            metrics_aggregation_fn=self.metrics_aggregation_fn,
        )
        self.context.step()
        return out

    def eval_step(self) -> Any:
        if self.context.topology.is_io_rank:
            assert self.dataloader_evaluation is not None, "needs an evaluation dataset on io ranks"
        return self.parallel_module.evaluation_step(
            dataloader=self.dataloader_evaluation, sync_batch_to_model_parallel=self.sync_batch_to_model_parallel,
            loss_function=self.loss_function, metrics_aggregation_fn=self.metrics_aggregation_fn,
        )

    def log_metrics(self, train_step_output: Any, eval_step_output: Any) -> dict[str, Any]:
        logger.info(f"completed step {self.context.iterations}")
        metrics: dict[str, Any] = {}
        if train_step_output.metrics:
            for k, v in train_step_output.metrics.items():
                metrics[f"training/{k}"] = v
        metrics["training/loss"] = train_step_output.loss
        metrics["training/step_duration"] = train_step_output.step_duration
        if train_step_output.global_grad_norm is not None:
            metrics["training/global_grad_norm"] = train_step_output.global_grad_norm
        if train_step_output.global_grad_norm_clipped is not None:
            metrics["training/global_grad_norm_clipped"] = train_step_output.global_grad_norm_clipped
        for name, lr in (train_step_output.learning_rates or {}).items():
            metrics[f"training/learning_rate_{name}"] = lr
        if train_step_output.overflow is not None:
            metrics["training/overflow"] = int(train_step_output.overflow)
        if train_step_output.no_overflow_steps is not None:
            metrics["training/no_overflow_steps"] = train_step_output.no_overflow_steps
        if train_step_output.current_loss_scale is not None:
            metrics["training/current_loss_scale"] = train_step_output.current_loss_scale
        if train_step_output.debug_dict:
            metrics.update(train_step_output.debug_dict)
        if eval_step_output is not None:
            for k, v in (eval_step_output.metrics or {}).items():
                metrics[f"evaluation/{k}"] = v
            metrics["evaluation/loss"] = eval_step_output.loss
            metrics["evaluation/step_duration"] = eval_step_output.step_duration
        logger.log_metrics(metrics, step=self.context.iterations)
        return metrics

    def _start_watchdog(self) -> Optional[HangWatchdog]:
        if not self.config.hang_watchdog_seconds:
            return None
        log_dir = getattr(getattr(self.context.config, "logger", None), "log_dir", None)
        return HangWatchdog(self.config.hang_watchdog_seconds, rank=self.context.topology.config.global_rank,
                            log_dir=log_dir, abort=self.config.hang_watchdog_abort)

    def run_training(self, return_metrics: bool = False) -> Optional[list[dict[str, Any]]]:
        out: list[dict[str, Any]] = []
        watchdog = self._start_watchdog()
        try:
            while self.context.iterations < (self.config.train_iterations or 0):
                tso = self.train_step()
                if (self.config.save_interval is not None and self.config.save_dir is not None
                        and self.context.iterations % self.config.save_interval == 0):
                    self.save_checkpoint()
                eso = None
                if self.config.eval_interval is not None and self.context.iterations % self.config.eval_interval == 0:
                    eso = self.eval_step()
                if self.context.topology.config.global_rank == 0:
                    m = self.log_metrics(tso, eso)
                    if return_metrics:
                        out.append(m)
                if watchdog is not None:
                    watchdog.heartbeat()
        finally:
            if watchdog is not None:
                watchdog.stop()
        return out if return_metrics else None


DeterminedBaseContextGeneric = TypeVar("DeterminedBaseContextGeneric", bound=DeterminedBaseContext)


class DeterminedBaseTrainer(BaseTrainer[DeterminedBaseContextGeneric, ParallelModuleGeneric]):
    """Trainer with Determined-cluster checkpoint storage and preemption (optional dependency).

    Without a Determined context (``context._use_determined`` False) it behaves exactly like
    ``BaseTrainer``.  With one it resumes from ``info.latest_checkpoint``, reports checkpoints and
    exits cleanly on preemption (reference ``trainer.py:317-558``).
    """

    def save_checkpoint(self, save_dir: Optional[Path] = None) -> Path:
        ctx = getattr(self.context, "determined_context", None)
        if not getattr(self.context, "_use_determined", False) or ctx is None:
            return super().save_checkpoint(save_dir)
        path = None
        if self.context.topology.config.global_rank == 0:
            metadata = {"steps_completed": self.context.iterations}
            with ctx.checkpoint.store_path(metadata) as (p, _storage_id):
                ctx.distributed.broadcast(str(p))
                path = Path(p)
                super().save_checkpoint(save_dir=path)
        else:
            path = Path(ctx.distributed.broadcast(None))
            super().save_checkpoint(save_dir=path)
        return path

    def run_training(self, return_metrics: bool = False) -> Optional[list[dict[str, Any]]]:
        ctx = getattr(self.context, "determined_context", None)
        if ctx is None:
            return super().run_training(return_metrics)
        out: list[dict[str, Any]] = []
        while self.context.iterations < (self.config.train_iterations or 0):
            tso = self.train_step()
            if self.config.save_interval is not None and self.context.iterations % self.config.save_interval == 0:
                self.save_checkpoint()
            eso = self.eval_step() if (self.config.eval_interval and self.context.iterations % self.config.eval_interval == 0) else None
            if self.context.topology.config.global_rank == 0:
                m = self.log_metrics(tso, eso)
                if return_metrics:
                    out.append(m)
            if ctx.preempt.should_preempt():
                self.save_checkpoint()
                if os.environ.get("DETERMINED_TEST") != "True":
                    raise SystemExit(0)
                break
        return out if return_metrics else None
