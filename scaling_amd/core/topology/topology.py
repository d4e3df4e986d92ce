"""Rank grid + process groups (Megatron "mpu" equivalent) on RCCL or gloo.

Parity: reference ``Topology`` (``src/scaling/core/topology/topology.py:20-441``).  The rank grid is
``arange(world).reshape(pp, dp, mp)`` — TP peers are adjacent ranks, which on an 8×MI355X node puts a
TP pair on one direct xGMI link.  Differences (MI355X-first):

* backend is ``nccl`` (= RCCL on ROCm) when a GPU is available, ``gloo`` otherwise (CPU CI), or
  whatever ``TopologyConfig.backend`` forces;
* rendezvous is env:// or tcp:// on the given master address;
* ``device_id`` is bound at init so RCCL communicators are created eagerly on the right device.
"""
from __future__ import annotations

import contextlib
import os
from datetime import timedelta
from typing import Any, Optional, TypedDict

import numpy as np
import torch
import torch.distributed as dist

from ..logging import logger
from .rng_tracker import CudaRNGStateTracker, RngTrackerState
from .topology_config import TopologyConfig


class TopologyState(TypedDict):
    model_parallel_constant_rng: RngTrackerState
    model_parallel_size: int
    pipe_parallel_size: int


class Topology:
    def __init__(self, config: TopologyConfig):
        self.config = config
        self.is_distributed_initialized = False
        assert config.world_size is not None and config.data_parallel_size is not None
        self._layout_3D = np.arange(config.world_size).reshape(
            config.pipe_parallel_size, config.data_parallel_size, config.model_parallel_size
        )
        rank = config.global_rank if config.global_rank is not None else 0
        where = np.argwhere(self._layout_3D == rank)
        assert len(where) == 1, f"global rank {rank} not in layout of world size {config.world_size}"
        self._pipe_parallel_rank, self._data_parallel_rank, self._model_parallel_rank = (int(x) for x in where[0])
        self._pipe_parallel_ranks: Optional[list[int]] = None
        self._data_parallel_ranks: Optional[list[int]] = None
        self._model_parallel_ranks: Optional[list[int]] = None
        self._pipe_parallel_group: Any = None
        self._data_parallel_group: Any = None
        self._model_parallel_group: Any = None
        self._device: Optional[torch.device] = None
        self._model_parallel_constant_rng: Optional[CudaRNGStateTracker] = None
        self.backend: Optional[str] = None

    # ------------------------------------------------------------------ rng
    @property
    def has_model_parallel_constant_rng(self) -> bool:
        return self._model_parallel_constant_rng is not None

    @property
    def model_parallel_constant_rng(self) -> Any:
        if self._model_parallel_constant_rng is None:
            return contextlib.nullcontext
        return self._model_parallel_constant_rng.fork

    def state_dict(self) -> Optional[TopologyState]:
        if self._model_parallel_constant_rng is None:
            return None
        return {
            "model_parallel_constant_rng": self._model_parallel_constant_rng.state_dict(),
            "model_parallel_size": self.config.model_parallel_size,
            "pipe_parallel_size": self.config.pipe_parallel_size,
        }

    def load_state_dict(self, state_dict: Optional[dict[str, Any]]) -> None:
        if self._model_parallel_constant_rng is None or state_dict is None:
            return
        if (
            self.config.model_parallel_size == state_dict["model_parallel_size"]
            and self.config.pipe_parallel_size == state_dict["pipe_parallel_size"]
        ):
            self._model_parallel_constant_rng.load_state_dict(state_dict["model_parallel_constant_rng"])

    # ------------------------------------------------------------------ init
    def initialize_device(self) -> None:
        rehearsal = self.config.backend == "gloo" and self.config.gloo_on_gpu
        if torch.cuda.is_available() and (self.config.backend != "gloo" or rehearsal):  # incl. "fake" (per-rank proxy)
            slot = self.config.local_slot if self.config.local_slot is not None else 0
            if rehearsal:
                slot %= torch.cuda.device_count()
            assert slot < torch.cuda.device_count(), (
                f"cannot assign gpu {slot} for {torch.cuda.device_count()} available gpus"
            )
            torch.cuda.set_device(slot)
            self._device = torch.device("cuda", slot)
        else:
            self._device = torch.device("cpu")

    def initialize_distributed(
        self,
        master_addr: str,
        master_port: str,
        torch_distributed_timeout_minutes: int = 20,
        seed: int = 42,
    ) -> None:
        assert not self.is_distributed_initialized, "distributed is already initialized"
        assert self.config.global_rank is not None, "cannot initialize distributed without global rank"
        logger.info(
            f"Topology.initialize_distributed() master {master_addr}:{master_port} "
            f"world_size {self.config.world_size} rank {self.config.global_rank}"
        )
        self.initialize_device()
        self._model_parallel_constant_rng = CudaRNGStateTracker(
            seed=seed + self.get_global_rank(model_parallel_rank=0), device=self.device
        )
        backend = self.config.backend or ("nccl" if self.device.type == "cuda" else "gloo")
        self.backend = backend
        if backend == "fake" and not dist.is_initialized():  # per-rank proxy: one process, stubbed collectives
            from .stub_collectives import init_fake_process_group, install as install_stubs

            assert self.config.pipe_parallel_size == 1, "the stubbed process group cannot run a pipeline"
            init_fake_process_group(self.config.world_size, self.config.global_rank)
            install_stubs()
        if not dist.is_initialized():
            kwargs: dict[str, Any] = dict(
                backend=backend,
                world_size=self.config.world_size,
                rank=self.config.global_rank,
                init_method=f"tcp://{master_addr}:{master_port}",
                timeout=timedelta(minutes=torch_distributed_timeout_minutes),
            )
            if backend == "nccl":
                kwargs["device_id"] = self.device
            dist.init_process_group(**kwargs)
        if backend == "gloo" and self.device.type == "cuda":  # 1-GPU rehearsal: make gloo stream-ordered
            from .gloo_gpu import install

            install()
        # every rank creates every group in the same order (collective requirement)
        for ranks in self.all_pipe_parallel_groups:
            g = dist.new_group(ranks)
            if self.config.global_rank in ranks:
                self._pipe_parallel_ranks, self._pipe_parallel_group = ranks, g
        for ranks in self.all_data_parallel_groups:
            g = dist.new_group(ranks)
            if self.config.global_rank in ranks:
                self._data_parallel_ranks, self._data_parallel_group = ranks, g
        for ranks in self.all_model_parallel_groups:
            g = dist.new_group(ranks)
            if self.config.global_rank in ranks:
                self._model_parallel_ranks, self._model_parallel_group = ranks, g
        self.is_distributed_initialized = True

    # ------------------------------------------------------------------ pipe
    @property
    def pipe_parallel_indices(self) -> list[int]:
        return list(range(self.config.pipe_parallel_size))

    @property
    def pipe_parallel_rank(self) -> int:
        return self._pipe_parallel_rank

    @property
    def previous_pipe_parallel_rank(self) -> Optional[int]:
        return None if self.is_first_pipe_parallel_rank else self.pipe_parallel_rank - 1

    @property
    def next_pipe_parallel_rank(self) -> Optional[int]:
        return None if self.is_last_pipe_parallel_rank else self.pipe_parallel_rank + 1

    @property
    def is_first_pipe_parallel_rank(self) -> bool:
        return self.pipe_parallel_rank == 0

    @property
    def is_last_pipe_parallel_rank(self) -> bool:
        return self.pipe_parallel_rank == self.config.pipe_parallel_size - 1

    @property
    def is_first_model_parallel_rank(self) -> bool:
        return self.model_parallel_rank == 0

    @property
    def is_io_rank(self) -> bool:
        return (self.is_first_pipe_parallel_rank or self.is_last_pipe_parallel_rank) and (
            self.is_first_model_parallel_rank
        )

    @property
    def pipe_parallel_ranks(self) -> list[int]:
        return self._pipe_parallel_ranks  # type: ignore[return-value]

    @property
    def pipe_parallel_group(self) -> Any:
        return self._pipe_parallel_group

    # ------------------------------------------------------------------ data
    @property
    def data_parallel_indices(self) -> list[int]:
        return list(range(self.config.data_parallel_size))

    @property
    def data_parallel_rank(self) -> int:
        return self._data_parallel_rank

    @property
    def data_parallel_ranks(self) -> list[int]:
        return self._data_parallel_ranks  # type: ignore[return-value]

    @property
    def data_parallel_group(self) -> Any:
        return self._data_parallel_group

    # ------------------------------------------------------------------ model
    @property
    def model_parallel_indices(self) -> list[int]:
        return list(range(self.config.model_parallel_size))

    @property
    def model_parallel_rank(self) -> int:
        return self._model_parallel_rank

    @property
    def model_parallel_ranks(self) -> list[int]:
        return self._model_parallel_ranks  # type: ignore[return-value]

    @property
    def model_parallel_group(self) -> Any:
        return self._model_parallel_group

    @property
    def device(self) -> torch.device:
        if self._device is None:
            raise RuntimeError("Device not specified")
        return self._device

    # ------------------------------------------------------------------ lookup
    def get_global_rank_group(
        self,
        pipe_parallel_rank: Optional[int] = None,
        data_parallel_rank: Optional[int] = None,
        model_parallel_rank: Optional[int] = None,
        flatten: bool = True,
    ) -> list[Any]:
        ranks = self._layout_3D
        if pipe_parallel_rank is not None:
            ranks = ranks[pipe_parallel_rank : pipe_parallel_rank + 1]
        if data_parallel_rank is not None:
            ranks = ranks[:, data_parallel_rank : data_parallel_rank + 1]
        if model_parallel_rank is not None:
            ranks = ranks[:, :, model_parallel_rank : model_parallel_rank + 1]
        return [int(r) for r in ranks.flatten()] if flatten else ranks.tolist()

    @property
    def all_pipe_parallel_groups(self) -> list[list[int]]:
        return [
            self.get_global_rank_group(data_parallel_rank=d, model_parallel_rank=m)
            for d in self.data_parallel_indices
            for m in self.model_parallel_indices
        ]

    @property
    def all_data_parallel_groups(self) -> list[list[int]]:
        return [
            self.get_global_rank_group(pipe_parallel_rank=p, model_parallel_rank=m)
            for p in self.pipe_parallel_indices
            for m in self.model_parallel_indices
        ]

    @property
    def all_model_parallel_groups(self) -> list[list[int]]:
        return [
            self.get_global_rank_group(pipe_parallel_rank=p, data_parallel_rank=d)
            for p in self.pipe_parallel_indices
            for d in self.data_parallel_indices
        ]

    def get_global_rank(
        self,
        pipe_parallel_rank: Optional[int] = None,
        data_parallel_rank: Optional[int] = None,
        model_parallel_rank: Optional[int] = None,
    ) -> int:
        p = self.pipe_parallel_rank if pipe_parallel_rank is None else pipe_parallel_rank
        d = self.data_parallel_rank if data_parallel_rank is None else data_parallel_rank
        m = self.model_parallel_rank if model_parallel_rank is None else model_parallel_rank
        return int(self._layout_3D[p, d, m])


def env_rank_info() -> dict[str, Any]:
    """torchrun / launcher env → (global_rank, world_size, local_slot)."""
    return dict(
        global_rank=int(os.environ.get("RANK", 0)),
        world_size=int(os.environ.get("WORLD_SIZE", 1)),
        local_slot=int(os.environ.get("LOCAL_SLOT", os.environ.get("LOCAL_RANK", 0))),
    )


def shutdown_distributed() -> None:
    """Every rank leaves together and tears its process group down before interpreter exit: a gloo rank that
    exits while a peer's transport threads still talk to it can abort that peer (std::terminate)."""
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
