"""DeepSpeed-style dynamic loss scaler (reference ``optimizer/loss_scaler.py:50-132``).

The overflow test is not done here per parameter (the reference syncs once per gradient); the
optimizer feeds the non-finite count that its fused L2/inf kernel already produced (one host sync
per step).
"""
from __future__ import annotations

from typing import Any, NamedTuple, Optional, TypedDict

import torch

from .loss_scaler_config import LossScalerConfig


class LossScalerState(TypedDict):
    current_scale: float
    current_hysteresis: float
    no_overflow_steps: int


class LossScalerOutput(NamedTuple):
    overflow: Optional[bool]
    no_overflow_steps: Optional[int]
    current_loss_scale: Optional[float]


class LossScaler:
    def __init__(self, config: LossScalerConfig, parameter_groups: Any = None) -> None:
        self.config = config
        self.parameter_groups = parameter_groups
        self._current_scale = config.initial_scale
        self._current_hysteresis = config.hysteresis
        self._no_overflow_steps = 0

    @property
    def current_scale(self) -> float:
        return self._current_scale if self.config.enable else 1.0

    def scale_loss(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self._current_scale if self.config.enable else loss

    def step(self, overflow: Optional[bool] = None) -> LossScalerOutput:
        if not self.config.enable:
            return LossScalerOutput(None, None, None)
        overflow = bool(overflow)
        if overflow:
            if self.config.hysteresis == 1 or self._current_hysteresis == 1:
                self._current_scale = max(self._current_scale / self.config.factor, self.config.min_scale)
            else:
                self._current_hysteresis -= 1
            self._no_overflow_steps = 0
        else:
            if self.config.consecutive_hysteresis:
                self._current_hysteresis = self.config.hysteresis
            if self._no_overflow_steps > 0 and self._no_overflow_steps % self.config.window == 0:
                if not self.config.consecutive_hysteresis:
                    self._current_hysteresis = self.config.hysteresis
                self._current_scale *= self.config.factor
            self._no_overflow_steps += 1
        return LossScalerOutput(overflow, self._no_overflow_steps, self._current_scale)

    def state_dict(self) -> LossScalerState:
        return {
            "current_scale": self._current_scale,
            "current_hysteresis": self._current_hysteresis,
            "no_overflow_steps": self._no_overflow_steps,
        }

    def load_state_dict(self, state: LossScalerState) -> None:
        self._current_scale = state["current_scale"]
        self._current_hysteresis = state["current_hysteresis"]
        self._no_overflow_steps = state["no_overflow_steps"]
