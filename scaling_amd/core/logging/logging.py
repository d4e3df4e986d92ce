"""Process-wide logger singleton.

Parity: reference ``src/scaling/core/logging/logging.py:46-209`` (``logger`` proxy, per-rank file
handler, JSON metric lines, optional TensorBoard/wandb/Determined sinks).  Optional sinks are
import-guarded: wandb/tensorboard/determined are not part of the MI355X image and are skipped when
absent instead of failing at import time.
"""
from __future__ import annotations

import json
import logging
import os
import socket
from typing import Any, Optional

from ..config import BaseConfig
from .logger_config import LoggerConfig, LogLevel

_COLORS = {
    logging.DEBUG: "\x1b[38;20m",
    logging.INFO: "\x1b[32;20m",
    logging.WARNING: "\x1b[33;20m",
    logging.ERROR: "\x1b[31;20m",
    logging.CRITICAL: "\x1b[31;1m",
}


class ColorFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        msg = super().format(record)
        if os.environ.get("NO_COLOR"):
            return msg
        return _COLORS.get(record.levelno, "") + msg + "\x1b[0m"


class Logger:
    def __init__(self, config: LoggerConfig, name: Optional[str] = None, global_rank: Optional[int] = None):
        self._tensorboard_writer: Any = None
        self._wandb: Any = None
        self._determined_context: Any = None
        self._logger = logging.getLogger("scaling-amd")
        self._logger.propagate = False
        for h in list(self._logger.handlers):
            self._logger.removeHandler(h)
        self._handler = logging.StreamHandler()
        self._logger.addHandler(self._handler)
        self._file_handler: Optional[logging.FileHandler] = None
        self.set_level(config.log_level)
        if config.log_dir is not None:
            config.log_dir.mkdir(exist_ok=True, parents=True)
            self._file_handler = logging.FileHandler(str(config.log_dir.absolute() / f"log_{name}.log"))
            self._logger.addHandler(self._file_handler)
            if config.use_tensorboard and config.is_rank_in_tensorboard_ranks(global_rank):
                try:
                    from torch.utils.tensorboard import SummaryWriter

                    self._tensorboard_writer = SummaryWriter(log_dir=str(config.log_dir / "tensorboard"))
                except ImportError:
                    self._logger.warning("tensorboard not installed; tensorboard logging disabled")
        if config.use_wandb and config.is_rank_in_wandb_ranks(global_rank):
            try:
                import wandb

                os.environ["WANDB_BASE_URL"] = config.wandb_host
                os.environ["WANDB_API_KEY"] = config.wandb_api_key or ""
                wandb.init(
                    project=config.wandb_project,
                    group=config.wandb_group,
                    name=f"{socket.gethostname()}-{global_rank}",
                    entity=config.wandb_team,
                )
                self._wandb = wandb
            except Exception:  # noqa: BLE001 - wandb is an optional sink
                self._logger.warning("wandb unavailable; wandb logging disabled")
        self._write_metrics = config.is_rank_in_metrics_ranks(global_rank)
        self._write_determined = config.is_rank_in_determined_metrics_ranks(global_rank)
        self.set_formatter(name)

    def set_level(self, log_level: LogLevel) -> None:
        self._logger.setLevel(log_level.name)
        self._handler.setLevel(log_level.name)

    def set_formatter(self, name: Optional[str] = None) -> None:
        fmt = "[%(asctime)s] [%(levelname)s] " + (f"[{name}] " if name is not None else "") + "%(message)s"
        self._handler.setFormatter(ColorFormatter(fmt))
        if self._file_handler is not None:
            self._file_handler.setFormatter(logging.Formatter(fmt))

    def configure_determined(self, determined_context: Any) -> None:
        self._determined_context = determined_context

    def log_metrics(self, metrics: dict[str, Any], step: int) -> None:
        if self._write_metrics:
            self.info(json.dumps(metrics))
        if self._wandb is not None:
            self._wandb.log(metrics, step=step)
        if self._tensorboard_writer is not None:
            for k, v in metrics.items():
                self._tensorboard_writer.add_scalar(k, v, step)
            self._tensorboard_writer.flush()
        if self._determined_context is not None and self._write_determined:
            train = {k: v for k, v in metrics.items() if not k.startswith("evaluation")}
            evaluation = {k: v for k, v in metrics.items() if k.startswith("evaluation")}
            if train:
                self._determined_context.train.report_training_metrics(steps_completed=step, metrics=train)
            if evaluation:
                self._determined_context.train.report_validation_metrics(steps_completed=step, metrics=evaluation)

    def log_config(self, config: BaseConfig) -> None:
        self.log_config_dict(config.as_dict())

    def log_config_dict(self, config_dict: dict) -> None:
        if self._wandb is not None:
            self._wandb.config.update(config_dict, allow_val_change=True)
        if self._tensorboard_writer is not None:
            for k, v in config_dict.items():
                self._tensorboard_writer.add_text(k, str(v))

    def debug(self, msg: object) -> None:
        self._logger.debug(msg)

    def info(self, msg: object) -> None:
        self._logger.info(msg)

    def warning(self, msg: object) -> None:
        self._logger.warning(msg)

    def error(self, msg: object) -> None:
        self._logger.error(msg)

    def critical(self, msg: object) -> None:
        self._logger.critical(msg)


DeterminedLogger = Logger


class _LoggerSingleton:
    def __init__(self) -> None:
        self._instance: Optional[Logger] = None

    def configure(self, config: LoggerConfig, name: Optional[str] = None, global_rank: Optional[int] = None) -> None:
        self._instance = Logger(config=config, name=name, global_rank=global_rank)

    def configure_determined(
        self, config: LoggerConfig, name: Optional[str] = None, global_rank: Optional[int] = None,
        determined_context: Any = None, **_: Any
    ) -> None:
        """Like ``configure``; metrics of the ranks in ``determined_metrics_ranks`` also go to the trial."""
        self.configure(config, name=name, global_rank=global_rank)
        assert self._instance is not None
        self._instance.configure_determined(determined_context)

    def __getattr__(self, item: str) -> Any:
        if self._instance is None:
            self._instance = Logger(LoggerConfig())
        return getattr(self._instance, item)


logger: Any = _LoggerSingleton()
