"""Logger config (field-compatible with reference ``src/scaling/core/logging/logger_config.py:21-126``)."""
from __future__ import annotations

import os
from datetime import datetime
from enum import Enum
from pathlib import Path
from typing import Any, Optional

from pydantic import Field, model_validator

from ..config import BaseConfig


class LogLevel(Enum):
    DEBUG = "debug"
    INFO = "info"
    WARNING = "warning"
    ERROR = "error"
    CRITICAL = "critical"


def is_date(string: str, fuzzy: bool = False) -> bool:
    try:
        from dateutil.parser import parse

        parse(string, fuzzy=fuzzy)
        return True
    except (ValueError, OverflowError):
        return False


def _in_ranks(rank: Optional[int], ranks: Optional[list[int]]) -> bool:
    if rank is None:
        return False
    return rank in ranks if ranks is not None else rank == 0


def get_wandb_api_from_env() -> Optional[str]:
    return os.getenv("WANDB_API_KEY")


class LoggerConfig(BaseConfig):
    log_level: LogLevel = Field(LogLevel.INFO, description="")
    log_dir: Optional[Path] = Field(None, description="")
    metrics_ranks: Optional[list[int]] = Field(
        None, description="global ranks that write metrics (None: rank 0 only)"
    )
    use_wandb: bool = Field(False, description="")
    wandb_ranks: Optional[list[int]] = Field(None, description="global ranks that write to wandb")
    wandb_host: str = Field("https://api.wandb.ai", description="url of the wandb host")
    wandb_team: str = Field("aleph-alpha", description="Team name for Weights and Biases.")
    wandb_project: str = Field("aleph-alpha-scaling", description="wandb project name")
    wandb_group: str = Field("debug", description="wandb group name")
    wandb_api_key: Optional[str] = Field(None, description="wandb api key")
    use_tensorboard: bool = Field(False, description="")
    tensorboard_ranks: Optional[list[int]] = Field(None, description="global ranks writing tensorboard")
    determined_metrics_ranks: Optional[list[int]] = Field(
        None, description="global ranks writing metrics to determined"
    )

    @model_validator(mode="before")
    @classmethod
    def add_dates_to_values(cls, values: dict[Any, Any]) -> dict[Any, Any]:
        stamp = datetime.now().strftime("%Y-%m-%d-%H-%M-%S")
        log_dir = values.get("log_dir")
        if log_dir is not None:
            log_dir = Path(log_dir)
            if not is_date(log_dir.name):
                values["log_dir"] = log_dir / stamp
        group = values.get("wandb_group")
        if group is not None and not is_date(group.split("-")[-1]):
            values["wandb_group"] = group + "-" + stamp
        return values

    @model_validator(mode="after")
    def check_if_api_key_is_provided_when_using_wandb(self) -> "LoggerConfig":
        key = self.wandb_api_key or get_wandb_api_from_env()
        if self.use_wandb and not key:
            raise ValueError("If 'use_wandb' is set to True a wandb api key needs to be provided.")
        if key != self.wandb_api_key:
            object.__setattr__(self, "wandb_api_key", key)
        return self

    def is_rank_in_tensorboard_ranks(self, rank: Optional[int]) -> bool:
        return _in_ranks(rank, self.tensorboard_ranks)

    def is_rank_in_wandb_ranks(self, rank: Optional[int]) -> bool:
        return _in_ranks(rank, self.wandb_ranks)

    def is_rank_in_metrics_ranks(self, rank: Optional[int]) -> bool:
        return _in_ranks(rank, self.metrics_ranks)

    def is_rank_in_determined_metrics_ranks(self, rank: Optional[int]) -> bool:
        return _in_ranks(rank, self.determined_metrics_ranks)
