"""Token store ``{prefix}.bin / .idx / .meta.json`` (format of reference ``core/data/memory_map.py``).

``.bin``: flat tokens of ``dtype``; ``.idx``: ``index_dtype`` pairs (start, length) per document;
``.meta.json``: ``{"dtype", "index_dtype", "document_count"}``.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Iterator, Literal, Optional

import numpy as np


class MemoryMapDataset:
    def __init__(self, prefix_path: Path, load_index_to_memory: bool = False) -> None:
        self.prefix_path = Path(prefix_path)
        self.load_index_to_memory = load_index_to_memory
        for f in (self.file_path_data, self.file_path_index, self.file_path_meta):
            assert f.is_file(), f"cannot initialize memory map, file not found: {f}"
        self.initialize()

    def initialize(self) -> None:
        meta = json.loads(self.file_path_meta.read_text())
        self.dtype = np.dtype(meta["dtype"])
        self.index_dtype = np.dtype(meta["index_dtype"])
        self.dtype_size = self.dtype.itemsize
        self.index_dtype_size = self.index_dtype.itemsize
        self.document_count = int(meta["document_count"])
        self._data = np.memmap(self.file_path_data, mode="r", order="C", dtype=self.dtype) if self.file_path_data.stat().st_size else np.zeros(0, self.dtype)
        idx = np.memmap(self.file_path_index, mode="r", order="C", dtype=self.index_dtype) if self.file_path_index.stat().st_size else np.zeros(0, self.index_dtype)
        self._index = idx[: 2 * self.document_count].reshape(self.document_count, 2)
        if self.load_index_to_memory:
            self._index = np.array(self._index)

    @property
    def file_path_data(self) -> Path:
        return Path(str(self.prefix_path) + ".bin")

    @property
    def file_path_index(self) -> Path:
        return Path(str(self.prefix_path) + ".idx")

    @property
    def file_path_meta(self) -> Path:
        return Path(str(self.prefix_path) + ".meta.json")

    def sizes(self, idx: Optional[int] = None) -> np.ndarray:
        if idx is None:
            return np.array(self._index[:, 1])
        return np.array(self._index[idx, 1], dtype=self.index_dtype)

    def __getitem__(self, idx: int) -> np.ndarray:
        if not isinstance(idx, (int, np.integer)):
            raise NotImplementedError
        assert idx < self.document_count, f"cannot retrieve document idx {idx} from {self.document_count} documents"
        start, size = (int(v) for v in self._index[idx])
        return self._data[start : start + size]

    def __len__(self) -> int:
        return self.document_count

    def __iter__(self) -> Iterator[np.ndarray]:
        for i in range(len(self)):
            yield self[i]


class MemoryMapDatasetBuilder(MemoryMapDataset):
    def __init__(
        self,
        prefix_path: Path,
        dtype: np.dtype = np.dtype(np.int32),
        index_dtype: np.dtype = np.dtype(np.int64),
    ):
        self.prefix_path = Path(prefix_path)
        self.dtype = np.dtype(dtype)
        self.index_dtype = np.dtype(index_dtype)
        self.initialize()

    def initialize(self) -> None:
        assert not self.file_path_data.is_file(), f"data file already exists: {self.file_path_data}"
        assert not self.file_path_index.is_file(), f"index file already exists: {self.file_path_index}"
        self.file_path_data.parent.mkdir(exist_ok=True, parents=True)
        self.data_file = open(self.file_path_data, "wb")
        self.index_file = open(self.file_path_index, "wb")
        self.current_index = 0
        self.document_count = 0

    def add(self, np_array: np.ndarray) -> None:
        assert len(np_array.shape) == 1, "cannot add arrays of more than one dimension"
        arr = np.asarray(np_array).astype(self.dtype)
        self.data_file.write(arr.tobytes(order="C"))
        self.index_file.write(np.array([self.current_index, len(arr)], dtype=self.index_dtype).tobytes(order="C"))
        self.current_index += len(arr)
        self.document_count += 1

    def finalize(self) -> None:
        assert not self.data_file.closed and not self.index_file.closed, "The Builder has been finalized already"
        self.data_file.close()
        self.index_file.close()
        with open(self.file_path_meta, "w") as f:
            json.dump(
                {"dtype": self.dtype.name, "index_dtype": self.index_dtype.name, "document_count": self.document_count},
                f,
            )

    def __enter__(self) -> "MemoryMapDatasetBuilder":
        return self

    def __exit__(self, *_args: object) -> Literal[False]:
        self.finalize()
        return False
