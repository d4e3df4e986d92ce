"""Megatron/fairseq indexed-dataset formats (reference ``transformer/data/legacy_dataset/indexed_dataset.py``).

* ``mmap`` ("MMIDIDX"): ``{prefix}.idx`` = magic ``MMIDIDX\\x00\\x00``, u64 version 1, u8 dtype code,
  u64 #items, u64 #docs, int32 sizes[#items], int64 byte pointers[#items], int64 doc_idx[#docs];
  ``{prefix}.bin`` = concatenated items.  Read through numpy memmaps (no copy).
* ``lazy`` / ``cached`` ("TNTIDX"): fairseq's older layout with element offsets; read-only support.
"""
from __future__ import annotations

import os
import struct
from typing import Any, Optional, Union

import numpy as np
import torch

DTYPES = {1: np.uint8, 2: np.int8, 3: np.int16, 4: np.int32, 5: np.int64, 6: np.float32, 7: np.float64, 8: np.uint16}
_CODES = {np.dtype(v): k for k, v in DTYPES.items()}
MMAP_MAGIC = b"MMIDIDX\x00\x00"
TNT_MAGIC = b"TNTIDX\x00\x00"


def code(dtype: Any) -> int:
    return _CODES[np.dtype(dtype)]


def index_file_path(prefix_path: str) -> str:
    return prefix_path + ".idx"


def data_file_path(prefix_path: str) -> str:
    return prefix_path + ".bin"


def best_fitting_dtype(vocab_size: Optional[int] = None) -> Any:
    return np.uint16 if vocab_size is not None and vocab_size < 65500 else np.int32


def infer_dataset_impl(path: str) -> Optional[str]:
    if not (os.path.exists(index_file_path(path)) and os.path.exists(data_file_path(path))):
        print(f"Dataset does not exist: {path}")
        return None
    with open(index_file_path(path), "rb") as f:
        magic = f.read(9)
    if magic[:8] == TNT_MAGIC:
        return "cached"
    if magic == MMAP_MAGIC:
        return "mmap"
    return None


class Index:
    """Reader of an MMIDIDX index file."""

    _HDR_MAGIC = MMAP_MAGIC

    def __init__(self, path: str, skip_warmup: bool = True) -> None:
        with open(path, "rb") as f:
            assert f.read(9) == MMAP_MAGIC, "Index file doesn't match expected format (MMIDIDX)"
            (version,) = struct.unpack("<Q", f.read(8))
            assert version == 1
            (dcode,) = struct.unpack("<B", f.read(1))
            self._dtype = np.dtype(DTYPES[dcode])
            self._len, self._doc_count = struct.unpack("<QQ", f.read(16))
            offset = f.tell()
        buf = np.memmap(path, mode="r", order="C")
        self._sizes = np.frombuffer(buf, dtype=np.int32, count=self._len, offset=offset)
        self._pointers = np.frombuffer(buf, dtype=np.int64, count=self._len, offset=offset + 4 * self._len)
        self._doc_idx = np.frombuffer(buf, dtype=np.int64, count=self._doc_count, offset=offset + 12 * self._len)
        self._buf = buf

    @staticmethod
    def write(path: str, dtype: Any, sizes: list[int], doc_idx: list[int]) -> None:
        sizes_a = np.asarray(sizes, dtype=np.int32)
        itemsize = np.dtype(dtype).itemsize
        pointers = np.zeros(len(sizes_a), dtype=np.int64)
        if len(sizes_a) > 1:
            np.cumsum(sizes_a[:-1].astype(np.int64) * itemsize, out=pointers[1:])
        with open(path, "wb") as f:
            f.write(MMAP_MAGIC)
            f.write(struct.pack("<Q", 1))
            f.write(struct.pack("<B", code(dtype)))
            f.write(struct.pack("<QQ", len(sizes_a), len(doc_idx)))
            f.write(sizes_a.tobytes(order="C"))
            f.write(pointers.tobytes(order="C"))
            f.write(np.asarray(doc_idx, dtype=np.int64).tobytes(order="C"))

    @property
    def dtype(self) -> np.dtype:
        return self._dtype

    @property
    def sizes(self) -> np.ndarray:
        return self._sizes

    @property
    def doc_idx(self) -> np.ndarray:
        return self._doc_idx

    def __getitem__(self, i: int) -> tuple[int, int]:
        return int(self._pointers[i]), int(self._sizes[i])

    def __len__(self) -> int:
        return self._len


class MMapIndexedDataset(torch.utils.data.Dataset):
    def __init__(self, path: str, skip_warmup: bool = True) -> None:
        super().__init__()
        self._do_init(path, skip_warmup)

    def _do_init(self, path: str, skip_warmup: bool) -> None:
        self._path = path
        self._index = Index(index_file_path(path), skip_warmup)
        self._bin = np.memmap(data_file_path(path), mode="r", order="C")

    def __getstate__(self) -> str:
        return self._path

    def __setstate__(self, state: str) -> None:
        self._do_init(state, True)

    def __len__(self) -> int:
        return len(self._index)

    def __getitem__(self, idx: Union[int, slice]) -> Union[np.ndarray, list[np.ndarray]]:
        if isinstance(idx, (int, np.integer)):
            ptr, size = self._index[int(idx)]
            return np.frombuffer(self._bin, dtype=self._index.dtype, count=size, offset=ptr)
        if isinstance(idx, slice):
            start, stop, step = idx.indices(len(self))
            if step != 1:
                raise ValueError("Slices into indexed_dataset must be contiguous")
            sizes = self._index.sizes[start:stop]
            flat = np.frombuffer(self._bin, dtype=self._index.dtype, count=int(sizes.sum()), offset=self._index[start][0])
            return np.split(flat, np.cumsum(sizes)[:-1])
        raise ValueError(f"idx needs to be of type int or slice, but is {type(idx)}.")

    def get(self, idx: int, offset: int = 0, length: Optional[int] = None) -> np.ndarray:
        ptr, size = self._index[idx]
        if length is None:
            length = size - offset
        return np.frombuffer(self._bin, dtype=self._index.dtype, count=length, offset=ptr + offset * self._index.dtype.itemsize)

    @property
    def sizes(self) -> np.ndarray:
        return self._index.sizes

    @property
    def doc_idx(self) -> np.ndarray:
        return self._index.doc_idx

    @staticmethod
    def exists(path: str) -> bool:
        return os.path.exists(index_file_path(path)) and os.path.exists(data_file_path(path))


class MMapIndexedDatasetBuilder:
    def __init__(self, out_file: str, dtype: Any = np.int64) -> None:
        self._data_file = open(out_file, "wb")
        self._dtype = np.dtype(dtype)
        self._sizes: list[int] = []
        self._doc_idx = [0]

    def add_item(self, tensor: Union[torch.Tensor, np.ndarray]) -> None:
        arr = np.asarray(tensor.numpy() if isinstance(tensor, torch.Tensor) else tensor, dtype=self._dtype)
        self._data_file.write(arr.tobytes(order="C"))
        self._sizes.append(arr.size)

    def end_document(self) -> None:
        self._doc_idx.append(len(self._sizes))

    def finalize(self, index_file: str) -> None:
        self._data_file.close()
        Index.write(index_file, self._dtype, self._sizes, self._doc_idx)


class IndexedDataset(torch.utils.data.Dataset):
    """fairseq "lazy" TNTIDX reader (element offsets, one file read per item)."""

    _HDR_MAGIC = TNT_MAGIC

    def __init__(self, path: str) -> None:
        super().__init__()
        self.path = path
        with open(index_file_path(path), "rb") as f:
            assert f.read(8) == TNT_MAGIC, "Index file doesn't match expected format (TNTIDX)"
            assert struct.unpack("<Q", f.read(8)) == (1,)
            dcode, self.element_size = struct.unpack("<QQ", f.read(16))
            self.dtype = np.dtype(DTYPES[dcode])
            self._len, self.s = struct.unpack("<QQ", f.read(16))
            (self.doc_count,) = struct.unpack("<Q", f.read(8))
            self.dim_offsets = np.fromfile(f, dtype=np.int64, count=self._len + 1)
            self.data_offsets = np.fromfile(f, dtype=np.int64, count=self._len + 1)
            self.sizes = np.fromfile(f, dtype=np.int64, count=self.s)
            self.doc_idx = np.fromfile(f, dtype=np.int64, count=self.doc_count)

    def __len__(self) -> int:
        return self._len

    def __getitem__(self, i: int) -> np.ndarray:
        if not 0 <= i < self._len:
            raise IndexError("index out of range")
        shape = self.sizes[self.dim_offsets[i] : self.dim_offsets[i + 1]]
        n = int(np.prod(shape))
        with open(data_file_path(self.path), "rb", buffering=0) as f:
            f.seek(int(self.data_offsets[i]) * self.element_size)
            return np.fromfile(f, dtype=self.dtype, count=n).reshape(shape)

    def size(self, index: int) -> int:
        return int(self.sizes[index])

    @staticmethod
    def exists(path: str) -> bool:
        return os.path.exists(index_file_path(path)) and os.path.exists(data_file_path(path))


class IndexedCachedDataset(IndexedDataset):
    """TNTIDX with the whole data file held in memory."""

    def __init__(self, path: str) -> None:
        super().__init__(path)
        self._data = np.fromfile(data_file_path(path), dtype=self.dtype)

    def __getitem__(self, i: int) -> np.ndarray:
        if not 0 <= i < self._len:
            raise IndexError("index out of range")
        shape = self.sizes[self.dim_offsets[i] : self.dim_offsets[i + 1]]
        a, b = int(self.data_offsets[i]), int(self.data_offsets[i + 1])
        return self._data[a:b].reshape(shape)


def make_builder(out_file: str, impl: str, vocab_size: Optional[int] = None) -> MMapIndexedDatasetBuilder:
    if impl != "mmap":
        raise NotImplementedError("only the mmap (MMIDIDX) format is written")
    return MMapIndexedDatasetBuilder(out_file, dtype=best_fitting_dtype(vocab_size))


def make_dataset(path: str, impl: str, skip_warmup: bool = False) -> Optional[torch.utils.data.Dataset]:
    if not IndexedDataset.exists(path):
        print(f"Dataset does not exist: {path}")
        return None
    if impl == "infer":
        impl = infer_dataset_impl(path) or ""
    if impl == "lazy":
        return IndexedDataset(path)
    if impl == "cached":
        return IndexedCachedDataset(path)
    if impl == "mmap":
        return MMapIndexedDataset(path, skip_warmup)
    print(f"Unknown dataset implementation: {impl}")
    return None


def get_indexed_dataset_(data_prefix: str, data_impl: str, skip_warmup: bool) -> Optional[torch.utils.data.Dataset]:
    return make_dataset(data_prefix, data_impl, skip_warmup)
