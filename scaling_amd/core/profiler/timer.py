"""Timers for the instruction profiler.

``SynchronizedTimer`` keeps the reference semantics (``src/scaling/core/profiler/timer.py:7``):
device synchronize on start/stop.  ``EventTimer`` is the MI355X-native default: it records HIP
events on the current stream, so profiling does not serialize the pipeline; durations are resolved
once per step at flush time.
"""
from __future__ import annotations

import time
from typing import Optional

import torch


def _sync() -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class SynchronizedTimer:
    def __init__(self) -> None:
        self.start_time: Optional[float] = None
        self.end_time: Optional[float] = None

    def start(self) -> None:
        _sync()
        self.start_time = time.time()

    def stop(self) -> None:
        assert self.start_time is not None, "timer has not been started and cannot be stopped"
        _sync()
        self.end_time = time.time()

    def reset(self) -> None:
        self.start_time = self.end_time = None

    def duration(self) -> float:
        assert self.start_time is not None and self.end_time is not None
        return self.end_time - self.start_time


class EventTimer:
    def __init__(self) -> None:
        self._gpu = torch.cuda.is_available()
        self._start: object = None
        self._end: object = None

    def start(self) -> None:
        if self._gpu:
            self._start = torch.cuda.Event(enable_timing=True)
            self._start.record()  # type: ignore[attr-defined]
        else:
            self._start = time.time()

    def stop(self) -> None:
        assert self._start is not None, "timer has not been started and cannot be stopped"
        if self._gpu:
            self._end = torch.cuda.Event(enable_timing=True)
            self._end.record()  # type: ignore[attr-defined]
        else:
            self._end = time.time()

    def reset(self) -> None:
        self._start = self._end = None

    def duration(self) -> float:
        assert self._start is not None and self._end is not None
        if self._gpu:
            self._end.synchronize()  # type: ignore[attr-defined]
            return self._start.elapsed_time(self._end) / 1000.0  # type: ignore[attr-defined]
        return float(self._end) - float(self._start)  # type: ignore[arg-type]
