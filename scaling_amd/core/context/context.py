"""Train/inference process context: config + topology + counters + RNG checkpointing.

Parity: reference ``BaseContext`` (``src/scaling/core/context/context.py:31-197``): same
``context_global_rank_{r}.pt`` file contents and the MAX all-reduce of counters on load when the
layout changed.  Works on CPU/gloo (no hard CUDA calls).
"""
from __future__ import annotations

import random
from pathlib import Path
from typing import Any, Optional, TypedDict, TypeVar

import numpy as np
import torch
import torch.distributed as dist

from ..config import BaseConfig
from ..topology import Topology, TopologyState
from ..utils.checkpoint_writer import save_file
from ..utils.safe_load import safe_load


class ContextState(TypedDict):
    iterations: int
    consumed_samples: int
    consumed_samples_evaluation: int
    random_rng_state: tuple
    np_rng_state: Any
    torch_rng_state: torch.Tensor
    torch_cuda_rng_state: Optional[torch.Tensor]
    topology: Optional[TopologyState]


class BaseContext:
    def __init__(self, config: BaseConfig, topology: Topology) -> None:
        self.config = config
        self.topology = topology
        self.iterations = 0
        self.consumed_samples = 0
        self.consumed_samples_evaluation = 0

    def initialize(
        self,
        master_addr: str,
        master_port: str,
        torch_distributed_timeout_minutes: int = 20,
        seed: int = 42,
        distributed: bool = True,
    ) -> None:
        if self.topology is not None:
            if distributed:
                self.topology.initialize_distributed(
                    master_addr=master_addr,
                    master_port=master_port,
                    torch_distributed_timeout_minutes=torch_distributed_timeout_minutes,
                    seed=seed,
                )
            else:
                self.topology.initialize_device()
            seed = seed + (self.topology.config.global_rank or 0)
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed(seed)

    def step(self) -> None:
        self.iterations += 1
        self.consumed_samples += self.topology.config.global_batch_size

    def state_dict(self) -> ContextState:
        return {
            "iterations": self.iterations,
            "consumed_samples": self.consumed_samples,
            "consumed_samples_evaluation": self.consumed_samples_evaluation,
            "random_rng_state": random.getstate(),
            "np_rng_state": np.random.get_state(),
            "torch_rng_state": torch.get_rng_state(),
            "torch_cuda_rng_state": torch.cuda.get_rng_state() if torch.cuda.is_available() else None,
            "topology": self.topology.state_dict(),
        }

    def load_state_dict(self, state_dict: dict[str, Any]) -> None:
        self.iterations = state_dict["iterations"]
        self.consumed_samples = state_dict["consumed_samples"]
        self.consumed_samples_evaluation = state_dict.get("consumed_samples_evaluation", 0)
        random.setstate(tuple(state_dict["random_rng_state"]))  # type: ignore[arg-type]
        np.random.set_state(state_dict["np_rng_state"])
        torch.set_rng_state(state_dict["torch_rng_state"])
        cuda_state = state_dict.get("torch_cuda_rng_state")
        if cuda_state is not None and torch.cuda.is_available():
            torch.cuda.set_rng_state(cuda_state)
        self.topology.load_state_dict(state_dict.get("topology"))

    def save_checkpoint(self, dir: Path | str) -> None:
        dir = Path(dir)
        if self.topology.config.global_rank == 0:
            self.config.save(dir / "config.yml")
        save_file(self.state_dict(), str(dir / f"context_global_rank_{self.topology.config.global_rank}.pt"))

    def load_checkpoint(self, dir: Path | str) -> None:
        dir = Path(dir)
        f = dir / f"context_global_rank_{self.topology.config.global_rank}.pt"
        if f.is_file():
            self.load_state_dict(safe_load(f))
        if self.topology.is_distributed_initialized:
            vals = [self.iterations, self.consumed_samples, self.consumed_samples_evaluation]
            if self.topology.config.global_rank != 0:
                vals = [0, 0, 0]
            t = torch.tensor(vals, dtype=torch.int64, device=self.topology.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            self.iterations, self.consumed_samples, self.consumed_samples_evaluation = (int(x) for x in t.tolist())


BaseContextGeneric = TypeVar("BaseContextGeneric", bound=BaseContext)


class DeterminedBaseContext(BaseContext):
    """BaseContext that also carries a Determined core context / profiler (optional dependency)."""

    def __init__(self, config: BaseConfig, topology: Topology) -> None:
        super().__init__(config=config, topology=topology)
        self.determined_context: Any = None
        self.determined_profiler: Any = None
        self._use_determined = False

    def initialize_with_determined(
        self,
        master_addr: str,
        master_port: str,
        determined_context: Any,
        determined_profiler: Any,
        torch_distributed_timeout_minutes: int = 20,
        seed: int = 42,
        distributed: bool = True,
    ) -> None:
        super().initialize(master_addr, master_port, torch_distributed_timeout_minutes, seed, distributed)
        self.determined_context = determined_context
        self.determined_profiler = determined_profiler
        self._use_determined = True
