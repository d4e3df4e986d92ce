"""Retrying file handle for flaky network filesystems (reference ``core/data/file_handles.py``):
``ESTALE`` / ``RetryableException`` are retried with exponential backoff (2^n s, max 32 s, 5 attempts)."""
from __future__ import annotations

import time
from errno import ESTALE
from pathlib import Path
from typing import IO, Any, Callable, Optional, TypeVar

V = TypeVar("V")


class RetryableException(Exception):
    pass


def is_retryable(e: BaseException) -> bool:
    if isinstance(e, OSError):
        return e.errno == ESTALE
    return isinstance(e, RetryableException)


class FileHandle:
    def __init__(self, path: Path, mode: str = "rb"):
        self._path = path
        self._mode = mode
        self._handle: Optional[IO[Any]] = None

    def retry_operation(self, func: Callable[[IO[Any]], V], max_attempts: int = 5, max_delay: int = 32) -> V:
        attempts = 0
        while True:
            try:
                if self._handle is None:
                    self._handle = open(self._path, self._mode)
                return func(self._handle)
            except Exception as e:  # noqa: BLE001
                if not is_retryable(e):
                    raise
                try:
                    self.close()
                except Exception as e_close:  # noqa: BLE001
                    print(f"Tried closing file {self._path} but it didn't work: {e_close}", flush=True)
                attempts += 1
                print(f"Caught retryable error for {self._path}: {e}. Attempt {attempts}/{max_attempts}.", flush=True)
                if attempts == max_attempts:
                    break
                time.sleep(min(2**attempts, max_delay))
        raise Exception(f"Stale file handle even after {attempts} retries for {self._path}.")

    def close(self) -> None:
        if self._handle is not None:
            self._handle.close()
            self._handle = None

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
