"""Model-parallel-constant RNG stream.

Same role as the reference ``CudaRNGStateTracker`` (``src/scaling/core/topology/rng_tracker.py:59-95``):
a generator state shared by all TP ranks so dropout in replicated regions matches.  Built only on public
torch APIs (``torch.cuda.get_rng_state/set_rng_state``) and works on CPU (gloo tests) as well.
HIP kernels that need randomness take an explicit Philox (seed, offset) pair drawn from this stream.
"""
from __future__ import annotations

import contextlib
from typing import Iterator, TypedDict

import torch


class RngTrackerState(TypedDict):
    seed: int
    state: torch.Tensor


class CudaRNGStateTracker:
    def __init__(self, seed: int, device: torch.device | None = None):
        self.seed = seed
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        )
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        self.state = gen.get_state()

    def _generator(self) -> torch.Generator:
        """The device's default generator, looked up once (``torch.cuda.get/set_rng_state`` re-resolve the device and
        go through a lazy-call closure on every use: a fork per dropout costs that four times per call)."""
        g = getattr(self, "_gen", None)
        if g is None:
            if self.device.type == "cuda":
                idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
                g = torch.cuda.default_generators[idx]
            else:
                g = torch.default_generator
            self._gen = g
        return g

    def _get(self) -> torch.Tensor:
        return self._generator().get_state()

    def _set(self, state: torch.Tensor) -> None:
        self._generator().set_state(state)

    def state_dict(self) -> RngTrackerState:
        return {"seed": self.seed, "state": self.state.clone().detach()}

    def load_state_dict(self, state_dict: RngTrackerState) -> None:
        self.seed = state_dict["seed"]
        self.state = state_dict["state"].clone()

    @contextlib.contextmanager
    def fork(self) -> Iterator[None]:
        orig = self._get()
        self._set(self.state)
        try:
            yield
        finally:
            self.state = self._get()
            self._set(orig)
