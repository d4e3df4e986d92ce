"""Blending of several datasets with an on-disk interleave index built by native C++.

Parity: reference ``core/data/blended_dataset.py:24-398``.  The index builder is
``scaling_amd._data.blended_sample`` (C++17, ``csrc/data/data_index.cpp``) replacing the Rust
``blended_dataset_loop`` wheel; file names and formats are unchanged
(``index_cache_blended_dataset_seed_{seed}_{ident}.{bin,meta.json,input.json}``).
"""
from __future__ import annotations

import hashlib
import json
import time
from pathlib import Path
from typing import Any, Generic, Optional, Sequence, TypeVar

import numpy as np
import torch

from ..logging import logger
from .base_dataset import BaseDataset, BaseDatasetBatchBeforeSyncGeneric, BaseDatasetBatchGeneric, BaseDatasetItemGeneric
from .blended_dataset_config import BlendedDatasetConfig

BaseDatasetGeneric = TypeVar("BaseDatasetGeneric", bound=BaseDataset)


def weights_by_num_docs(examples: list[int], alpha: float = 0.3) -> np.ndarray:
    e = np.array(examples, np.float64)
    p = e / e.sum()
    q = p**alpha
    q = q / q.sum()
    w = q / p
    return w / w.sum()


def weights_examples_proportional(examples: list[int], temperature: float = 1.0, maximum: Optional[float] = None) -> np.ndarray:
    assert temperature is not None and temperature != 0, "temperature must be a non-zero float"
    e = np.array(examples, np.float64)
    p = e / e.sum()
    if maximum:
        assert maximum > 0, f"examples-proportional sampling requires maximum limit > 0 (current max = {maximum})"
        e[e > maximum] = maximum
    q = e / e.sum()
    if temperature != 1.0:
        q = q ** (1.0 / temperature)
        q = q / q.sum()
    w = q / p
    return w / w.sum()


def native_blended_sample(counts: np.ndarray, stem: str) -> int:
    from scaling_amd import _data  # type: ignore[attr-defined]

    return int(_data.blended_sample(np.asarray(counts, dtype=np.int64), stem))


class BaseBlendedDataset(
    Generic[BaseDatasetItemGeneric, BaseDatasetBatchBeforeSyncGeneric, BaseDatasetBatchGeneric, BaseDatasetGeneric],
    BaseDataset[BaseDatasetItemGeneric, BaseDatasetBatchBeforeSyncGeneric, BaseDatasetBatchGeneric],
):
    def __init__(self, seed: int, config: BlendedDatasetConfig, datasets: Sequence[BaseDatasetGeneric]) -> None:
        self.config = config
        self.datasets = datasets
        self.num_datasets = len(datasets)
        self.seed: Optional[int] = None
        self.random_index: Optional[np.ndarray] = None
        self.weights = np.ones(self.num_datasets) / self.num_datasets
        self.set_seed(seed=seed, shuffle=True)

    def ident(self) -> str:
        prefix = "-".join(d.ident() for d in self.datasets)
        weights = "-".join(str(round(w * 100) / 100) for w in self.weights.tolist())
        ph = hashlib.md5(prefix.encode("utf-8")).hexdigest()
        wh = hashlib.md5(weights.encode("utf-8")).hexdigest()
        return f"{self.datasets[0].__class__.__name__}_prefix_{ph}_weights_{wh}"

    def get_data_index_cache_filename_stem(self, seed: int) -> str:
        assert self.config.cache_directory is not None, "cache directory is needed"
        self.config.cache_directory.mkdir(exist_ok=True, parents=True)
        return str(self.config.cache_directory / f"index_cache_blended_dataset_seed_{seed}_{self.ident()}")

    def get_data_index_cache_filename_meta(self, seed: int) -> str:
        return self.get_data_index_cache_filename_stem(seed) + ".meta.json"

    def get_data_index_cache_filename_input(self, seed: int) -> str:
        return self.get_data_index_cache_filename_stem(seed) + ".input.json"

    def get_data_index_cache_filename_bin(self, seed: int) -> str:
        return self.get_data_index_cache_filename_stem(seed) + ".bin"

    def __len__(self) -> int:
        return max(self.size, self.config.minimum_dataset_size)

    def __getitem__(self, index: int) -> BaseDatasetItemGeneric:
        if self.size < self.config.minimum_dataset_size:
            index %= self.size
        if self.num_datasets > 1 and self.random_index is not None:
            index = int(self.random_index[index])
        if self.num_datasets == 1:
            return self.datasets[0][index]
        ds, i = self.dataset_indices[index]
        return self.datasets[int(ds)][int(i)]

    def _counts(self, docs: list[int]) -> np.ndarray:
        rel = self.weights / self.weights.max()
        if self.config.weight_examples_proportional:
            return np.array([max(1, int(round(p * n))) for n, p in zip(docs, rel)], dtype=np.int64)
        return np.array([max(1, int(p * n)) for n, p in zip(docs, rel)], dtype=np.int64)

    def set_seed(self, seed: int, shuffle: bool = True) -> None:
        if seed == self.seed:
            return
        self.seed = seed
        assert shuffle, "Blended datasets should always be shuffled"
        if self.num_datasets == 1:
            self.datasets[0].set_seed(seed=seed, shuffle=shuffle)
            self.size = len(self.datasets[0])
            return
        docs = []
        for ds in self.datasets:
            ds.set_seed(seed=seed, shuffle=shuffle)
            docs.append(len(ds))
        if self.config.weight_by_num_documents:
            if self.config.weight_examples_proportional:
                self.weights = weights_examples_proportional(docs, self.config.ep_temperature, self.config.ep_maximum)
            else:
                self.weights = weights_by_num_docs(docs, self.config.weighted_sampler_alpha)
        else:
            assert self.config.weights is not None and len(self.config.weights) == len(self.datasets)
            w = np.array(self.config.weights, dtype=np.float64)
            assert w.sum() > 0.0
            self.weights = w / w.sum()
        stem = self.get_data_index_cache_filename_stem(seed)
        meta, inp, binf = (stem + ".meta.json", stem + ".input.json", stem + ".bin")
        is_rank0 = (not torch.distributed.is_initialized()) or torch.distributed.get_rank() == 0
        if not Path(meta).is_file() and is_rank0:
            t0 = time.time()
            native_blended_sample(self._counts(docs), stem)
            logger.info(f"{self.__class__.__name__} blended index for seed {seed} built in {time.time() - t0:.2f}s")
        attempts = 0
        while not (Path(binf).is_file() and Path(inp).is_file() and Path(meta).is_file()):
            attempts += 1
            if attempts % 12 == 0:
                logger.info(f"BlendedDataset waiting on index for seed {seed}; elapsed {attempts * 5 / 60} minutes")
            time.sleep(5)
        self.dataset_meta = json.loads(Path(meta).read_text())
        shape = tuple(self.dataset_meta["shape"])
        dtype = np.dtype(self.dataset_meta["dtype"])
        if self.config.load_dataset_indices_to_memory:
            self.dataset_indices = np.fromfile(binf, dtype=dtype).reshape(shape)
        else:
            self.dataset_indices = np.memmap(binf, mode="r", order="C", dtype=dtype, shape=shape)
        self.size = shape[0]
        if self.config.load_dataset_indices_to_memory:
            if self.config.shuffle_dataset_indices and shuffle:
                np.random.RandomState(seed=seed).shuffle(self.dataset_indices)
            self.random_index = None
        else:
            ri = np.arange(self.size)
            if self.config.shuffle_dataset_indices and shuffle:
                np.random.RandomState(seed=seed).shuffle(ri)
            self.random_index = ri

    def collate(self, batch: list[BaseDatasetItemGeneric]) -> BaseDatasetBatchBeforeSyncGeneric:
        return self.datasets[0].collate(batch=batch)

    @staticmethod
    def sync_batch_to_model_parallel(topology: Any, batch: Any) -> Any:
        raise NotImplementedError

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}_{self.datasets[0].__class__.__name__}"
