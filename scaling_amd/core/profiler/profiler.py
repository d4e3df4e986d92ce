"""Per-instruction pipeline profiler writing the reference ``profile.json`` schema.

Parity: reference ``Profiler`` (``src/scaling/core/profiler/profiler.py:24-139``) — timers keyed by
(timer_name, micro_batch_id, buffer_id), active for steps [start, start+profile_steps), gathered to
rank 0.  MI355X-native: HIP-event timing by default and roctx ranges around every instruction so a
``rocprofv3 --marker-trace`` run shows the pipeline schedule.
"""
from __future__ import annotations

import collections
import json
from contextlib import contextmanager
from typing import Any, Generator, NamedTuple, Optional

import torch
import torch.distributed as dist

from ..topology import Topology
from .profiler_config import ProfilerConfig
from .timer import EventTimer, SynchronizedTimer


def _roctx_push(name: str) -> None:
    try:
        torch.cuda.nvtx.range_push(name)  # maps to roctx on ROCm builds
    except Exception:  # noqa: BLE001
        pass


def _roctx_pop() -> None:
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:  # noqa: BLE001
        pass


class ProfilerObservation(NamedTuple):
    timer_name: str
    step: int
    micro_batch_id: int
    buffer_id: int
    pipe_parallel_rank: int
    data_parallel_rank: int
    model_parallel_rank: int
    duration: float


class Profiler:
    def __init__(self, config: ProfilerConfig, topology: Topology) -> None:
        self.config = config
        self.topology = topology
        self.steps = 0
        self.step_save = 0
        self.end_step = config.profile_start_at_step + config.profile_steps
        self.enabled = config.profile_steps > 0 and config.profiler_output is not None
        self.observations: list[ProfilerObservation] = []
        self.timers: Any = {}
        self._timer_cls = EventTimer if config.use_events else SynchronizedTimer

    def _active(self) -> bool:
        return self.enabled and self.config.profile_start_at_step <= self.steps <= self.end_step

    def step(self) -> None:
        self.steps += 1
        cls = self._timer_cls
        self.timers = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(cls)))

    def flush(self) -> None:
        if not self.enabled:
            return
        for name, per_mb in self.timers.items():
            for mb, per_buf in per_mb.items():
                for buf, timer in per_buf.items():
                    self.observations.append(
                        ProfilerObservation(
                            timer_name=name,
                            step=self.step_save,
                            micro_batch_id=mb,
                            buffer_id=buf,
                            pipe_parallel_rank=self.topology.pipe_parallel_rank,
                            data_parallel_rank=self.topology.data_parallel_rank,
                            model_parallel_rank=self.topology.model_parallel_rank,
                            duration=timer.duration(),
                        )
                    )
        self.step_save += 1
        if self.steps == self.end_step:
            self.save()

    def save(self) -> None:
        if self.config.profiler_output is None:
            return
        gathered: Optional[list] = None
        if dist.is_initialized():
            gathered = [None] * self.topology.config.world_size if self.topology.config.global_rank == 0 else None
            dist.gather_object(self.observations, gathered, dst=0)
        else:
            gathered = [self.observations]
        if self.topology.config.global_rank in (0, None):
            obs = [o for lst in (gathered or []) for o in (lst or [])]
            self.config.profiler_output.parent.mkdir(exist_ok=True, parents=True)
            with open(self.config.profiler_output, "w", encoding="UTF-8") as f:
                json.dump(
                    {
                        "pipe_parallel_size": self.topology.config.pipe_parallel_size,
                        "data_parallel_size": self.topology.config.data_parallel_size,
                        "model_parallel_size": self.topology.config.model_parallel_size,
                        "gradient_accumulation_steps": self.topology.config.gradient_accumulation_steps,
                        "observations": [o._asdict() for o in obs],
                    },
                    f,
                    indent=4,
                )

    def start_timer(self, timer_name: str, micro_batch_id: Optional[int], buffer_id: Optional[int]) -> None:
        if self._active():
            self.timers[timer_name][micro_batch_id][buffer_id].start()

    def stop_timer(self, timer_name: str, micro_batch_id: Optional[int], buffer_id: Optional[int]) -> None:
        if self._active():
            self.timers[timer_name][micro_batch_id][buffer_id].stop()

    @contextmanager
    def time(
        self, timer_name: str, micro_batch_id: Optional[int], buffer_id: Optional[int]
    ) -> Generator[None, None, None]:
        active = self._active()
        if active:
            _roctx_push(f"{timer_name}/mb{micro_batch_id}/buf{buffer_id}")
        self.start_timer(timer_name, micro_batch_id, buffer_id)
        try:
            yield
        finally:
            self.stop_timer(timer_name, micro_batch_id, buffer_id)
            if active:
                _roctx_pop()
