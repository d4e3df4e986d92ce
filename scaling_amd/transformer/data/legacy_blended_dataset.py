"""Blend of legacy (MMIDIDX) text datasets (reference ``transformer/data/legacy_blended_dataset.py``).

Sampling stops as soon as ANY dataset has delivered its quota (the legacy semantics; the current
``BaseBlendedDataset`` runs until every dataset is complete).  Index stored as an int32 MMIDIDX file of
(dataset, index) pairs plus a ``.done`` marker.
"""
from __future__ import annotations

import hashlib
import heapq
import time
from pathlib import Path
from typing import Any, Optional

import numpy as np
import torch

from ...core import BaseBlendedDataset, BlendedDatasetConfig
from ...core.data.blended_dataset import weights_by_num_docs
from .legacy_dataset import get_indexed_dataset_
from .legacy_dataset.indexed_dataset import Index
from .text_dataset import TextDataset
from .text_dataset_batch import TextDatasetBatch, TextDatasetBatchBeforeSync
from .text_dataset_item import TextDatasetItem


def weights_examples_proportional(number_of_examples_by_dataset: list[int], temperature: float = 1.0,
                                  maximum: Any = None) -> np.ndarray:
    """T5 examples-proportional mixing with an optional per-dataset or global rate limit K."""
    assert temperature is not None and temperature != 0, "expect a non-zero temperature"
    e = np.array(number_of_examples_by_dataset, np.float64)
    p = e / e.sum()
    if maximum:
        if isinstance(maximum, list):
            lim = np.array(maximum, np.float64)
            e = np.where(e > lim, lim, e)
        else:
            assert maximum > 0, f"examples-proportional sampling requires maximum limit > 0 (current max = {maximum})"
            e[e > maximum] = maximum
    q = e / e.sum()
    if temperature != 1.0:
        q = q ** (1.0 / temperature)
        q = q / q.sum()
    w = q / p
    return w / w.sum()


def legacy_blend(counts: np.ndarray) -> np.ndarray:
    """(dataset, index) rows: repeatedly sample the dataset furthest behind its quota (lowest index on
    ties) until the first dataset completes."""
    counts = np.asarray(counts, dtype=np.int64)
    heap = [(0.0, i) for i in range(len(counts))]
    sampled = np.zeros(len(counts), dtype=np.int64)
    out = []
    while True:
        _, i = heapq.heappop(heap)
        out.append((i, int(sampled[i])))
        sampled[i] += 1
        if sampled[i] >= counts[i]:
            break
        heapq.heappush(heap, (sampled[i] / counts[i], i))
    return np.array(out, dtype=np.int32).reshape(-1, 2)


class LegacyBlendedDataset(BaseBlendedDataset[TextDatasetItem, TextDatasetBatchBeforeSync, TextDatasetBatch, TextDataset]):
    def __init__(self, seed: int, config: BlendedDatasetConfig, datasets: list[TextDataset], shuffle: bool = True):
        self.config = config
        self.datasets = datasets
        self.num_datasets = len(datasets)
        self.dataset_indices_: Any = None
        self.size = 0
        self.ep_maximum_dict: Optional[dict] = None
        self.weights = np.array(config.weights if config.weights is not None else [1.0] * self.num_datasets, np.float64)
        self.seed: Optional[int] = None
        self.set_seed(seed, shuffle=shuffle)

    def get_data_index_cache_filename_stem(self, seed: int) -> str:
        assert self.config.cache_directory is not None, "cache directory is needed"
        Path(self.config.cache_directory).mkdir(exist_ok=True, parents=True)
        prefixes = "-".join(Path(d.data_prefix).name for d in self.datasets)
        weights = "-".join(str(round(w * 100) / 100) for w in self.weights.tolist())
        ph = hashlib.md5(prefixes.encode("utf-8")).hexdigest()
        wh = hashlib.md5(weights.encode("utf-8")).hexdigest()
        return str(Path(self.config.cache_directory) /
                   f"index_cache_blended_dataset_seed_{seed}_seq_len_{self.datasets[0].sequence_length}_prefix_{ph}_weights_{wh}")

    def set_seed(self, seed: int, shuffle: bool = True) -> None:
        assert shuffle, "Blended datasets should always be shuffled"
        if seed == self.seed:
            return
        self.seed = seed
        if self.num_datasets == 1:
            self.datasets[0].set_seed(seed)
            self.size = len(self.datasets[0])
            return
        docs = []
        for ds in self.datasets:
            ds.compute_data_index(seed=seed)
            docs.append(len(ds))
        cfg = self.config
        if cfg.weight_by_num_documents:
            if cfg.weight_examples_proportional:
                limits: Any = cfg.ep_maximum
                if self.ep_maximum_dict is not None:
                    limits = [self.ep_maximum_dict.get(Path(d.data_prefix).stem, cfg.ep_maximum or n)
                              for d, n in zip(self.datasets, docs)]
                self.weights = weights_examples_proportional(docs, cfg.ep_temperature, limits)
            else:
                self.weights = weights_by_num_docs(docs, cfg.weighted_sampler_alpha)
        else:
            w = np.array(self.weights, dtype=np.float64)
            assert w.sum() > 0.0
            self.weights = w / w.sum()
        stem = self.get_data_index_cache_filename_stem(seed)
        done = stem + ".done"
        is_rank0 = (not torch.distributed.is_initialized()) or torch.distributed.get_rank() == 0
        if not Path(done).is_file() and is_rank0:
            rel = self.weights / self.weights.max()
            rnd = round if cfg.weight_examples_proportional else int
            counts = np.array([max(1, int(rnd(p * n))) for n, p in zip(docs, rel)], dtype=np.int64)
            rows = legacy_blend(counts)
            rows.tofile(stem + ".bin")
            Index.write(stem + ".idx", np.int32, [2] * len(rows), [0])
            Path(done).write_text("True")
        while not (Path(stem + ".bin").is_file() and Path(stem + ".idx").is_file() and Path(done).is_file()):
            time.sleep(0.5)
        self.dataset_indices_ = get_indexed_dataset_(stem, "mmap", True)
        self.size = len(self.dataset_indices_)

    def __len__(self) -> int:
        return max(self.size, self.config.minimum_dataset_size)

    def __getitem__(self, idx: int) -> TextDatasetItem:
        if self.size < self.config.minimum_dataset_size:
            idx %= self.size
        if self.num_datasets == 1:
            return self.datasets[0][idx]
        ds, i = (int(v) for v in self.dataset_indices_[idx])
        return self.datasets[ds][i]
