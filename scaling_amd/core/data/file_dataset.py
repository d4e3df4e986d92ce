"""Memory-map-format dataset read with seek/read instead of mmap (SIGBUS-free on network FS).

Same files as ``MemoryMapDataset``; every file operation goes through ``FileHandle.retry_operation``
(reference ``core/data/file_dataset.py:11-196``).
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import IO, Any, Iterator, Optional

import numpy as np

from .file_handles import FileHandle


def retry_array_from_file(handle: FileHandle, dtype: np.dtype, count: int, offset: int) -> np.ndarray:
    def op(f: IO[Any]) -> np.ndarray:
        f.seek(offset)
        arr = np.fromfile(f, dtype=dtype, count=count)
        if len(arr) != count:
            from .file_handles import RetryableException

            raise RetryableException(f"short read: expected {count} got {len(arr)}")
        return arr

    return handle.retry_operation(op)


class FileDataset:
    def __init__(self, prefix_path: Path, load_index_to_memory: bool = False) -> None:
        self.prefix_path = Path(prefix_path)
        self.load_index_to_memory = load_index_to_memory
        self.initialize()

    def initialize(self) -> None:
        meta_file = FileHandle(self.file_path_meta, "r")
        meta = meta_file.retry_operation(json.load)
        meta_file.close()
        self.dtype = np.dtype(meta["dtype"])
        self.index_dtype = np.dtype(meta["index_dtype"])
        self.dtype_size = self.dtype.itemsize
        self.index_dtype_size = self.index_dtype.itemsize
        self.document_count = int(meta["document_count"])
        self._bin_file = FileHandle(self.file_path_data, "rb")
        self._index_file = FileHandle(self.file_path_index, "rb")
        self._index: Optional[np.ndarray] = None
        if self.load_index_to_memory:
            self._index = retry_array_from_file(
                self._index_file, self.index_dtype, 2 * self.document_count, 0
            ).reshape(self.document_count, 2)
            self._index_file.close()

    @property
    def file_path_data(self) -> Path:
        return Path(str(self.prefix_path) + ".bin")

    @property
    def file_path_index(self) -> Path:
        return Path(str(self.prefix_path) + ".idx")

    @property
    def file_path_meta(self) -> Path:
        return Path(str(self.prefix_path) + ".meta.json")

    def _entry(self, idx: int) -> tuple[int, int]:
        if self._index is not None:
            s, n = self._index[idx]
            return int(s), int(n)
        s, n = retry_array_from_file(self._index_file, self.index_dtype, 2, int(idx * 2) * self.index_dtype_size)
        return int(s), int(n)

    def sizes(self, idx: Optional[int] = None) -> np.ndarray:
        if idx is None:
            if self._index is not None:
                return np.array(self._index[:, 1])
            all_idx = retry_array_from_file(self._index_file, self.index_dtype, 2 * self.document_count, 0)
            return all_idx.reshape(-1, 2)[:, 1].copy()
        return np.array(self._entry(idx)[1], dtype=self.index_dtype)

    def __getitem__(self, idx: int) -> np.ndarray:
        assert idx < self.document_count, f"cannot retrieve document idx {idx} from {self.document_count} documents"
        start, size = self._entry(int(idx))
        return retry_array_from_file(self._bin_file, self.dtype, size, start * self.dtype_size)

    def __len__(self) -> int:
        return self.document_count

    def __iter__(self) -> Iterator[np.ndarray]:
        for i in range(len(self)):
            yield self[i]

    def __del__(self) -> None:
        for n in ("_bin_file", "_index_file"):
            h = getattr(self, n, None)
            if h is not None:
                h.close()
