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

from ..utils.checkpoint_writer import checkpoint_writer
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
        self._unpublished: Optional[tuple[Path, int]] = None  # async checkpoint written but not yet 'latest'
        checkpoint_writer.configure(config.async_checkpointing)
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
        """Writes ``global_step<N>/`` and points ``latest`` at it.  With ``async_checkpointing`` the files are
        written by a background thread and ``latest`` moves at the next ``flush_checkpoints`` (next save or end
        of training), once every rank's files are complete."""
        self.flush_checkpoints()
        save_dir = Path(save_dir or self.config.save_dir)  # type: ignore[arg-type]
        it_dir = save_dir / f"global_step{self.context.iterations}"
        it_dir.mkdir(exist_ok=True, parents=True)
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        self.parallel_module.save_checkpoint(it_dir, separate_file_for_parameters=self.config.separate_file_for_parameters)
        self.optimizer.save_checkpoint(it_dir)
        self.context.save_checkpoint(it_dir)
        if checkpoint_writer.async_mode:
            self._unpublished = (save_dir, self.context.iterations)
            logger.info(f"checkpoint {it_dir} queued for writing")
            return save_dir
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        self._publish(save_dir, self.context.iterations)
        logger.info(f"saved checkpoint: {it_dir}")
        return save_dir

    def _publish(self, save_dir: Path, iterations: int) -> None:
        if self.context.topology.config.global_rank == 0:
            tmp = save_dir / "latest.tmp"
            with open(tmp, "w", encoding="UTF-8") as f:
                f.write(f"global_step{iterations}")
            os.replace(tmp, save_dir / "latest")

    def flush_checkpoints(self) -> None:
        """Waits for this rank's queued checkpoint files, then (all ranks) publishes the checkpoint as ``latest``."""
        if self._unpublished is None:
            checkpoint_writer.wait()
            return
        save_dir, iterations = self._unpublished
        self._unpublished = None
        checkpoint_writer.wait()
        if torch.distributed.is_initialized():
            torch.distributed.barrier()
        self._publish(save_dir, iterations)
        logger.info(f"saved checkpoint: {save_dir / f'global_step{iterations}'}")

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
            self.flush_checkpoints()
        finally:
            if watchdog is not None:
                watchdog.stop()
        return out if return_metrics else None


DeterminedBaseContextGeneric = TypeVar("DeterminedBaseContextGeneric", bound=DeterminedBaseContext)


class DeterminedBaseTrainer(BaseTrainer[DeterminedBaseContextGeneric, ParallelModuleGeneric]):
    """Trainer with Determined-cluster checkpoint storage and preemption (optional dependency).

    Without a Determined context (``context._use_determined`` False) it behaves exactly like
    ``BaseTrainer``.  With one (reference ``trainer.py:317-558``) it
    * resumes from the trial's ``latest_checkpoint`` (pause/resume of an experiment), forcing optimizer
      and context state to load;
    * stores checkpoints through ``checkpoint.store_path`` and, with ``delete_past_optimizer_states``,
      removes the optimizer-state files of every older completed checkpoint of the trial;
    * on construction (rank 0) deletes checkpoints written off the ``save_interval`` grid (preemption
      saves), keeping the newest one for resuming;
    * saves and exits when the cluster asks for preemption, and advances the profiler agent per step.

    The cluster is reached only through ``_cluster_info`` and ``_trial_checkpoints`` (objects with the
    Determined API's ``uuid``/``metadata``/``state``/``delete``/``remove_files``), so the logic runs and
    is tested against duck-typed stand-ins where ``determined`` is not installed.
    """

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        if self.context.topology.config.global_rank == 0 and self._use_determined():
            self.delete_preempted_checkpoints_determined()

    # ------------------------------------------------------------------ cluster access (overridable)
    def _use_determined(self) -> bool:
        return bool(getattr(self.context, "_use_determined", False)) and getattr(self.context, "determined_context", None) is not None

    def _cluster_info(self) -> Any:
        try:
            import determined as det  # type: ignore
        except ImportError:
            return None
        return det.get_cluster_info()

    def _trial_checkpoints(self) -> list[Any]:
        """Checkpoints of this trial, oldest (lowest batch number) first."""
        import determined as det  # type: ignore
        from determined.experimental import client  # type: ignore

        info = self._cluster_info()
        assert info is not None
        trial = client.get_trial(info.trial.trial_id)
        return list(trial.get_checkpoints(sort_by=det.experimental.client.CheckpointSortBy.BATCH_NUMBER,
                                          order_by=det.experimental.client.CheckpointOrderBy.ASC))

    @staticmethod
    def _completed(ckpt: Any) -> bool:
        st = getattr(ckpt, "state", None)
        return str(getattr(st, "name", st)).upper().endswith("COMPLETED")

    # ------------------------------------------------------------------ checkpoints
    def save_checkpoint(self, save_dir: Optional[Path] = None) -> Path:
        if not self._use_determined():
            return super().save_checkpoint(save_dir)
        ctx = self.context.determined_context
        if self.context.topology.config.global_rank == 0:
            metadata = {"steps_completed": self.context.iterations}
            with ctx.checkpoint.store_path(metadata) as (p, storage_id):
                ctx.distributed.broadcast(str(p))
                path = Path(p)
                super().save_checkpoint(save_dir=path)
                self.flush_checkpoints()  # the storage context uploads on exit: files must be complete
            if self.config.delete_past_optimizer_states:
                self.delete_previous_optimizer_states_determined(str(storage_id))
        else:
            path = Path(ctx.distributed.broadcast(None))
            super().save_checkpoint(save_dir=path)
            self.flush_checkpoints()
        return path

    def load_checkpoint(self, load_dir: Optional[Path] = None, load_optimizer_states: bool = True,
                        load_context: bool = True, allowed_missing_keys_in_checkpoint: Optional[list[str]] = None,
                        allowed_unexpected_keys_in_checkpoint: Optional[list[str]] = None,
                        ignore_keys_in_checkpoint: Optional[list[str]] = None) -> bool:
        kw = dict(allowed_missing_keys_in_checkpoint=allowed_missing_keys_in_checkpoint,
                  allowed_unexpected_keys_in_checkpoint=allowed_unexpected_keys_in_checkpoint,
                  ignore_keys_in_checkpoint=ignore_keys_in_checkpoint)
        info = self._cluster_info() if self._use_determined() else None
        latest = getattr(info, "latest_checkpoint", None) if info is not None else None
        if latest is not None:
            # a paused / preempted trial continues exactly where it stopped
            with self.context.determined_context.checkpoint.restore_path(latest) as path:
                logger.info(f"Updating load checkpoint directory from {load_dir} to {path} according to determined")
                return super().load_checkpoint(load_dir=Path(path), load_optimizer_states=True, load_context=True, **kw)
        return super().load_checkpoint(load_dir=load_dir, load_optimizer_states=load_optimizer_states,
                                       load_context=load_context, **kw)

    def delete_preempted_checkpoints_determined(self) -> list[str]:
        """Deletes checkpoints saved off the ``save_interval`` grid except the newest; returns their uuids."""
        if os.environ.get("DETERMINED_TEST") == "True":
            return []
        deleted: list[str] = []
        try:
            ckpts = self._trial_checkpoints()
            for c in ckpts[:-1]:  # the newest stays: a paused trial resumes from it
                steps = int(c.metadata["steps_completed"])
                if self.config.save_interval and steps % self.config.save_interval != 0:
                    logger.warning(f"Delete determined checkpoint {c.uuid} at step {steps} - likely saved at preemption")
                    c.delete()
                    deleted.append(str(c.uuid))
        except Exception as ex:  # noqa: BLE001 - cluster API failures must not stop training
            logger.error(f"deletion of previous determined preempted checkpoints failed, will not delete anything: {ex}")
        return deleted

    def delete_previous_optimizer_states_determined(self, latest_uuid: str) -> list[str]:
        """Removes ``optimizer_state*`` files from every completed checkpoint but ``latest_uuid`` (rank 0)."""
        if os.environ.get("DETERMINED_TEST") == "True" or self.context.topology.config.global_rank != 0:
            return []
        cleaned: list[str] = []
        try:
            for c in self._trial_checkpoints():
                if str(c.uuid) != latest_uuid and self._completed(c):
                    logger.info(f"Requesting optimizer states deletion of ckpt {c.uuid}")
                    c.remove_files(["global_step*/*optimizer_state*pt"])
                    cleaned.append(str(c.uuid))
        except Exception as ex:  # noqa: BLE001
            logger.error(f"deletion of previous optimizer states failed, will not delete anything: {ex}")
            logger.error(f"DET_ENV_VARS_AFTER_FAILURE: { {k: v for k, v in os.environ.items() if k.startswith('DET_')} }")
        return cleaned

    # ------------------------------------------------------------------ loop
    def run_training(self, return_metrics: bool = False) -> Optional[list[dict[str, Any]]]:
        if not self._use_determined():
            return super().run_training(return_metrics)
        ctx = self.context.determined_context
        profiler = getattr(self.context, "determined_profiler", None)
        out: list[dict[str, Any]] = []
        while self.context.iterations < (self.config.train_iterations or 0):
            if profiler is not None:
                profiler.update_batch_idx(self.context.iterations)
            tso = self.train_step()
            if ctx.preempt.should_preempt():
                self.save_checkpoint()
                print("exiting program after preemption.", flush=True)
                if os.environ.get("DETERMINED_TEST") != "True":
                    raise SystemExit(0)
                break
            if self.config.save_interval is not None and self.context.iterations % self.config.save_interval == 0:
                self.save_checkpoint()
            eso = self.eval_step() if (self.config.eval_interval and self.context.iterations % self.config.eval_interval == 0) else None
            if self.context.topology.config.global_rank == 0:
                m = self.log_metrics(tso, eso)
                if return_metrics:
                    out.append(m)
        return out if return_metrics else None
