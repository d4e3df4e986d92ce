"""Host-side hang watchdog (SURVEY §5.3 "MI355X plan").

A daemon thread expects a heartbeat at least every ``timeout_s`` seconds (the trainer beats once per step).
When a step stalls — typically a rank stuck in an RCCL collective whose peer died, or a kernel that never
drains — it dumps every Python thread's stack (``faulthandler``) to stderr and to ``<log_dir>/hang_rank<r>.txt``
and, with ``abort=True``, ends the process with exit code 124 so the launcher's fail-fast tears the job down
instead of leaving it hanging until the collective timeout (20 min by default).
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from pathlib import Path
from typing import Callable, Optional, TextIO


class HangWatchdog:
    def __init__(self, timeout_s: float, rank: int = 0, log_dir: Optional[Path] = None, abort: bool = False,
                 on_hang: Optional[Callable[[float], None]] = None, poll_s: Optional[float] = None) -> None:
        assert timeout_s > 0
        self.timeout_s = float(timeout_s)
        self.rank = rank
        self.log_dir = Path(log_dir) if log_dir is not None else None
        self.abort = abort
        self.on_hang = on_hang
        self.fired = 0
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._poll = poll_s if poll_s is not None else min(5.0, self.timeout_s / 4)
        self._thread = threading.Thread(target=self._run, name=f"hang-watchdog-rank{rank}", daemon=True)
        self._thread.start()

    def heartbeat(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=2 * self._poll + 1)

    def _dump(self, stalled: float, stream: TextIO) -> None:
        stream.write(f"[hang-watchdog] rank {self.rank}: no progress for {stalled:.0f}s (timeout {self.timeout_s:.0f}s); "
                     f"stacks of all threads:\n")
        stream.flush()
        faulthandler.dump_traceback(file=stream, all_threads=True)
        stream.flush()

    def _run(self) -> None:
        while not self._stop.wait(self._poll):
            stalled = time.monotonic() - self._last
            if stalled < self.timeout_s:
                continue
            self.fired += 1
            self._dump(stalled, sys.stderr)
            if self.log_dir is not None:
                try:
                    self.log_dir.mkdir(parents=True, exist_ok=True)
                    with open(self.log_dir / f"hang_rank{self.rank}.txt", "a") as f:
                        self._dump(stalled, f)
                except OSError:
                    pass
            if self.on_hang is not None:
                self.on_hang(stalled)
            if self.abort:
                os._exit(124)
            self._last = time.monotonic()  # report again after another full timeout
