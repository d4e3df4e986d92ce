"""Pipeline schedule base: dependency-aware replay (``illustrate``), PNG rendering (``visualize``) and a
profile replay simulator.  Behaviour follows reference ``pipeline_schedule/base.py:14-697`` (same
DEPENDENCY_MAP semantics, same ``profile.json`` schema); rendering/simulation code is independent.
"""
from __future__ import annotations

import collections
import json
from abc import ABC, abstractmethod
from pathlib import Path
from typing import Any, Optional

from PIL import Image, ImageDraw

from ...topology import Topology, TopologyConfig
from .instructions import InstructionBase

DEPENDENCY_MAP = {
    "InstructionRecvActivation": {"instruction": "InstructionSendActivation", "previous": True},
    "InstructionSendActivation": {"instruction": "InstructionRecvActivation", "previous": False},
    "InstructionRecvGrad": {"instruction": "InstructionSendGrad", "previous": False},
    "InstructionSendGrad": {"instruction": "InstructionRecvGrad", "previous": True},
}

COLORS = {
    "InstructionLoadMicroBatch": (120, 120, 120),
    "InstructionForwardPass": (66, 133, 244),
    "InstructionBackwardPass": (234, 67, 53),
    "InstructionLoss": (251, 188, 5),
    "InstructionSendActivation": (52, 168, 83),
    "InstructionRecvActivation": (52, 168, 83),
    "InstructionSendGrad": (171, 71, 188),
    "InstructionRecvGrad": (171, 71, 188),
    "InstructionReduceTiedGrads": (0, 172, 193),
    "InstructionOptimizerStep": (0, 0, 0),
}


def _short(name: str) -> str:
    return name.replace("Instruction", "")


class PipelineScheduleBase(ABC):
    def __init__(self, topology: Topology):
        self.topology = topology

    @abstractmethod
    def instructions(self) -> list[InstructionBase]:
        pass

    @abstractmethod
    def required_buffer_count(self) -> int:
        pass

    def _valid_micro_batch(self, micro_batch_id: int) -> bool:
        return 0 <= micro_batch_id < self.topology.config.gradient_accumulation_steps

    def _is_valid_pipe_parallel_rank(self, rank: Optional[int]) -> bool:
        return rank is not None and 0 <= rank < self.topology.config.pipe_parallel_size

    @classmethod
    def _all_rank_instructions(cls, gradient_accumulation_steps: int, pipe_parallel_size: int) -> dict[int, list]:
        out = {}
        for rank in range(pipe_parallel_size):
            topo = Topology(
                TopologyConfig(  # type: ignore[call-arg]
                    global_rank=rank,
                    pipe_parallel_size=pipe_parallel_size,
                    gradient_accumulation_steps=gradient_accumulation_steps,
                    model_parallel_size=1,
                    data_parallel_size=1,
                    micro_batch_size=1,
                )
            )
            out[rank] = cls(topology=topo).instructions()
        return out

    @classmethod
    def illustrate(cls, gradient_accumulation_steps: int, pipe_parallel_size: int) -> dict[str, Any]:
        """Lock-step replay: a rank executes its next instruction once its p2p partner is at the matching one."""
        queues = {r: collections.deque(ins) for r, ins in
                  cls._all_rank_instructions(gradient_accumulation_steps, pipe_parallel_size).items()}
        steps: list[dict[int, Optional[dict[str, Any]]]] = []
        P = pipe_parallel_size
        while any(queues.values()):
            heads = {r: (q[0] if q else None) for r, q in queues.items()}
            ready = {}
            for r, ins in heads.items():
                if ins is None:
                    ready[r] = False
                    continue
                if ins.name == "InstructionReduceTiedGrads":
                    ready[r] = all(h is not None and h.name == "InstructionReduceTiedGrads" for h in heads.values())
                elif ins.name in DEPENDENCY_MAP:
                    dep = DEPENDENCY_MAP[ins.name]
                    peer = (r - 1) % P if dep["previous"] else (r + 1) % P
                    ready[r] = heads[peer] is not None and heads[peer].name == dep["instruction"]
                else:
                    ready[r] = True
            if not any(ready.values()):
                raise RuntimeError("pipeline schedule deadlock in illustrate()")
            step: dict[int, Optional[dict[str, Any]]] = {}
            for r in range(P):
                if ready[r]:
                    step[r] = {"name": queues[r].popleft().name}
                else:
                    step[r] = None
            steps.append(step)
        idle = {r: sum(1 for s in steps if s[r] is None) for r in range(P)}
        total = sum(idle.values())
        return {
            "steps": steps,
            "count_idling": idle,
            "pct_idling": {r: c / len(steps) for r, c in idle.items()},
            "count_idling_total": total,
            "pct_idling_total": total / (len(steps) * P),
        }

    @classmethod
    def visualize(cls, gradient_accumulation_steps: int, pipe_parallel_size: int, cell: int = 12) -> Image.Image:
        ill = cls.illustrate(gradient_accumulation_steps, pipe_parallel_size)
        steps = ill["steps"]
        w, h = max(1, len(steps)) * cell, pipe_parallel_size * cell
        img = Image.new("RGB", (w, h + 14), (255, 255, 255))
        d = ImageDraw.Draw(img)
        for t, step in enumerate(steps):
            for r, cmd in step.items():
                if cmd is None:
                    continue
                d.rectangle([t * cell, r * cell, (t + 1) * cell - 1, (r + 1) * cell - 1], fill=COLORS.get(cmd["name"], (200, 200, 200)))
        d.text((2, h + 1), f"pp={pipe_parallel_size} acc={gradient_accumulation_steps} idle={ill['pct_idling_total']:.1%}", fill=(0, 0, 0))
        return img

    # ------------------------------------------------------------------ profile replay
    @classmethod
    def load_profile(cls, profile_file: Path) -> dict[str, Any]:
        return json.loads(Path(profile_file).read_text())

    @classmethod
    def visualize_profile(
        cls, profile_file: Path, milliseconds_per_pixel: float = 1.0, pipe_pixels: int = 40
    ) -> tuple[dict[str, Any], Image.Image]:
        sim = SimulationEngine(cls.load_profile(profile_file), schedule_cls=cls)
        timings = sim.simulate()
        return timings, sim.render(milliseconds_per_pixel, pipe_pixels)


class SimulationEngine:
    """Replays measured per-instruction durations on the ideal schedule.

    p2p wait is removed by charging each Send/Recv pair min(send, recv) (reference
    ``base.py:365-418``); computes per-stage busy/idle time for one step (averaged over the data-
    and model-parallel ranks recorded in the profile).
    """

    def __init__(self, profile: dict[str, Any], schedule_cls: Any):
        self.profile = profile
        self.schedule_cls = schedule_cls
        self.pp = int(profile["pipe_parallel_size"])
        self.acc = int(profile["gradient_accumulation_steps"])
        dur: dict[tuple, list[float]] = collections.defaultdict(list)
        for o in profile["observations"]:
            key = (o["timer_name"], o["pipe_parallel_rank"], o["micro_batch_id"])
            dur[key].append(float(o["duration"]))
        self.duration = {k: sum(v) / len(v) for k, v in dur.items()}
        self.events: list[tuple[int, str, float, float]] = []

    def _d(self, name: str, rank: int, mb: Optional[int]) -> float:
        short = _short(name)
        for key in ((short, rank, mb), (name, rank, mb), (short, rank, None), (name, rank, None)):
            if key in self.duration:
                return self.duration[key]
        return 0.0

    def simulate(self) -> dict[str, Any]:
        per_rank = self.schedule_cls._all_rank_instructions(self.acc, self.pp)
        queues = {r: collections.deque(v) for r, v in per_rank.items()}
        clock = {r: 0.0 for r in range(self.pp)}
        busy = {r: 0.0 for r in range(self.pp)}
        self.events = []
        P = self.pp
        guard = 0
        while any(queues.values()):
            guard += 1
            if guard > 10_000_000:
                raise RuntimeError("simulation did not terminate")
            progressed = False
            for r in range(P):
                if not queues[r]:
                    continue
                ins = queues[r][0]
                if ins.name in DEPENDENCY_MAP:
                    dep = DEPENDENCY_MAP[ins.name]
                    peer = (r - 1) % P if dep["previous"] else (r + 1) % P
                    if not queues[peer] or queues[peer][0].name != dep["instruction"]:
                        continue
                    pins = queues[peer][0]
                    t0 = max(clock[r], clock[peer])
                    d = min(self._d(ins.name, r, ins.micro_batch_id), self._d(pins.name, peer, pins.micro_batch_id))
                    for rr, ii in ((r, ins), (peer, pins)):
                        self.events.append((rr, ii.name, t0, t0 + d))
                        busy[rr] += d
                        clock[rr] = t0 + d
                        queues[rr].popleft()
                    progressed = True
                elif ins.name == "InstructionReduceTiedGrads":
                    if all(q and q[0].name == "InstructionReduceTiedGrads" for q in queues.values()):
                        t0 = max(clock.values())
                        for rr in range(P):
                            d = self._d(queues[rr][0].name, rr, None)
                            self.events.append((rr, "InstructionReduceTiedGrads", t0, t0 + d))
                            busy[rr] += d
                            clock[rr] = t0 + d
                            queues[rr].popleft()
                        progressed = True
                else:
                    d = self._d(ins.name, r, ins.micro_batch_id)
                    self.events.append((r, ins.name, clock[r], clock[r] + d))
                    busy[r] += d
                    clock[r] += d
                    queues[r].popleft()
                    progressed = True
            if not progressed:
                raise RuntimeError("simulation deadlock")
        total = max(clock.values()) if clock else 0.0
        return self.summarize(total, busy)

    def summarize(self, total: float, busy: dict[int, float]) -> dict[str, Any]:
        return {
            "total_time": total,
            "busy_time": busy,
            "idle_time": {r: total - b for r, b in busy.items()},
            "pct_idling": {r: (total - b) / total if total > 0 else 0.0 for r, b in busy.items()},
        }

    def render(self, milliseconds_per_pixel: float, pipe_pixels: int) -> Image.Image:
        total = max((e[3] for e in self.events), default=0.0)
        width = max(1, int(total * 1000 / milliseconds_per_pixel) + 1)
        width = min(width, 20000)
        scale = width / max(total, 1e-12)
        img = Image.new("RGB", (width, self.pp * pipe_pixels), (255, 255, 255))
        d = ImageDraw.Draw(img)
        for r, name, t0, t1 in self.events:
            x0, x1 = int(t0 * scale), max(int(t0 * scale), int(t1 * scale) - 1)
            d.rectangle([x0, r * pipe_pixels, x1, (r + 1) * pipe_pixels - 1], fill=COLORS.get(name, (200, 200, 200)))
        return img
