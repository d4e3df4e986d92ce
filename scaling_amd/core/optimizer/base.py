from abc import ABC, abstractmethod
from pathlib import Path
from typing import Any, NamedTuple, Optional, TypedDict

import torch


class OptimizerStepOutput(NamedTuple):
    global_grad_norm: Optional[float]
    global_grad_norm_clipped: Optional[float]
    learning_rates: Optional[dict[str, float]]
    overflow: Optional[bool]
    no_overflow_steps: Optional[int]
    current_loss_scale: Optional[float]
    debug_dict: Optional[dict[str, float]]


class BaseOptimizerState(TypedDict):
    pass


class BaseOptimizer(ABC):
    def __init__(self, config: Any) -> None:
        pass

    def __repr__(self) -> str:
        return self.__class__.__name__

    @abstractmethod
    def step(self) -> OptimizerStepOutput: ...

    @abstractmethod
    def backward(self, loss: torch.Tensor) -> None: ...

    def log_state(self) -> None:
        pass

    @abstractmethod
    def state_dict(self) -> Any: ...

    @abstractmethod
    def save_checkpoint(self, dir: Path) -> None: ...

    @abstractmethod
    def load_checkpoint(self, dir: Path) -> None: ...

    @abstractmethod
    def refresh_optimizer_after_model_change(self) -> None: ...

    # hooks used by the pipeline engine to overlap the gradient reduction with the last backward
    def prepare_grad_sync(self) -> None:
        pass

    def finish_grad_sync(self) -> None:
        pass

    # hooks used by the engine to overlap the ZeRO parameter all-gather with the next forward pass
    def attach_param_sync(self, layers: Any) -> None:
        pass

    def wait_param_sync(self, layer: Optional[Any] = None) -> None:
        pass

    def wait_grad_zeroing(self) -> None:
        """Makes the current stream wait for an asynchronous gradient zeroing (overlapped step); default no-op."""
        return None
