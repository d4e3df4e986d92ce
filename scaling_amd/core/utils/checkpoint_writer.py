"""Checkpoint file writer: synchronous (the reference's behaviour) or asynchronous.

A 7B checkpoint is ~13 GB of weights plus ~80 GB of fp32 optimizer state; ``torch.save`` of that to a network
file system stalls every rank for minutes.  With ``TrainerConfig.async_checkpointing`` the training thread only
snapshots the state to host memory (device-to-host copies, after which the GPU state may change) and queues the
files; one background thread serialises and writes them (``<file>.tmp`` then an atomic rename) while training
continues.  The file set and formats are exactly those of a synchronous save.

Publishing: the ``latest`` pointer of a checkpoint must name a step whose files are complete on EVERY rank, and
the writer thread may not issue collectives.  So a checkpoint is published at the next synchronisation point of
the training thread: the next ``save_checkpoint`` and the end of training call ``wait`` (this rank's files are
on disk), then a barrier, then rank 0 writes ``latest`` (``BaseTrainer.flush_checkpoints``).  A job that dies in
between resumes from the previous complete checkpoint.
"""
from __future__ import annotations

import copy
import os
import queue
import threading
from pathlib import Path
from typing import Any, Optional, Union

import torch


def _snapshot(obj: Any) -> Any:
    """Deep copy with every tensor moved to (unshared) host memory.  Mappings become plain dicts (a ``defaultdict``
    or other dict subclass cannot always be rebuilt from pairs, and ``torch.save`` needs no subclass), named tuples
    keep their type, and mutable non-tensor leaves (sets, objects) are deep-copied so later training-state
    mutation cannot leak into a queued file."""
    if isinstance(obj, torch.Tensor):
        t = obj.detach()
        return t.to("cpu", copy=True) if t.device.type != "cpu" else t.clone()
    if isinstance(obj, dict):
        return {k: _snapshot(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_snapshot(v) for v in obj]
    if isinstance(obj, tuple):
        items = [_snapshot(v) for v in obj]
        return type(obj)(*items) if hasattr(obj, "_fields") else tuple(items)
    if obj is None or isinstance(obj, (bool, int, float, complex, str, bytes, Path)):
        return obj
    return copy.deepcopy(obj)


class CheckpointWriter:
    def __init__(self) -> None:
        self.async_mode = False
        self._queue: "queue.Queue[Optional[tuple[Any, str]]]" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self._pending = 0
        self._cv = threading.Condition()

    def configure(self, async_mode: bool) -> None:
        self.wait()
        self.async_mode = bool(async_mode)

    def save(self, obj: Any, path: Union[str, Path]) -> None:
        path = str(path)
        if not self.async_mode:
            torch.save(obj, path)
            return
        snap = _snapshot(obj)
        self._ensure_thread()
        with self._cv:
            self._pending += 1
        self._queue.put((snap, path))

    def _ensure_thread(self) -> None:
        if self._thread is None or not self._thread.is_alive():
            self._thread = threading.Thread(target=self._run, name="checkpoint-writer", daemon=True)
            self._thread.start()

    def _run(self) -> None:
        while True:
            job = self._queue.get()
            if job is None:
                return
            obj, path = job
            try:
                tmp = path + ".tmp"
                torch.save(obj, tmp)
                os.replace(tmp, path)
            except BaseException as e:  # surfaced by wait() on the training thread
                self._error = e
            finally:
                del obj
                with self._cv:
                    self._pending -= 1
                    self._cv.notify_all()

    @property
    def pending(self) -> int:
        return self._pending

    def wait(self) -> None:
        """Blocks until every queued file is on disk; re-raises a write error."""
        with self._cv:
            while self._pending > 0:
                self._cv.wait()
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError("asynchronous checkpoint write failed") from e


checkpoint_writer = CheckpointWriter()


def save_file(obj: Any, path: Union[str, Path]) -> None:
    """``torch.save`` through the process-wide checkpoint writer (async when the trainer enabled it)."""
    checkpoint_writer.save(obj, path)
