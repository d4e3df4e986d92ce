"""Pre-tokenized text dataset over a memory map (reference ``transformer/data/text_dataset.py``).

Items are exactly ``sequence_length + 1`` tokens packed from shuffled documents (last token of a
chunk is re-used as first token of the next).  The packing index is built by native C++
(``scaling_amd._data.text_index``) from the same numpy ``RandomState(seed)`` document order as the
reference, and stored in the same on-disk format (``{stem}.bin/.idx/.meta.json`` memory map of
int64 ``(doc, start, end)`` triples).
"""
from __future__ import annotations

import hashlib
import json
import os
import time
from pathlib import Path
from typing import Optional, Union

import numpy as np
import torch

from ...core import BaseBlendedDataset, BaseDataset, FileDataset, MemoryMapDataset, MemoryMapDatasetBuilder, Topology, broadcast_data
from .text_dataset_batch import TextDatasetBatch, TextDatasetBatchBeforeSync
from .text_dataset_item import TextDatasetItem


def _rank() -> int:
    return torch.distributed.get_rank() if torch.distributed.is_initialized() else 0


def write_text_index(stem: str, doc_sizes: np.ndarray, doc_order: np.ndarray, sequence_length: int,
                     only_full_sequences: bool, allow_incomplete_sequences_every_n: int) -> int:
    """Builds the packing index natively and writes it as an int64 memory map; returns the item count."""
    from scaling_amd import _data  # type: ignore[attr-defined]

    flat, pairs = _data.text_index(np.ascontiguousarray(doc_sizes, dtype=np.int64),
                                   np.ascontiguousarray(doc_order, dtype=np.int64), int(sequence_length),
                                   bool(only_full_sequences), int(allow_incomplete_sequences_every_n))
    for suffix in (".bin", ".idx", ".meta.json"):
        if Path(stem + suffix).is_file():
            Path(stem + suffix).unlink()
    tmp = f".tmp{os.getpid()}"
    flat.astype(np.int64).tofile(stem + ".bin")
    pairs.astype(np.int64).tofile(stem + ".idx")
    n = len(pairs) // 2
    with open(stem + ".meta.json" + tmp, "w") as f:
        json.dump({"dtype": "int64", "index_dtype": "int64", "document_count": n}, f)
    os.replace(stem + ".meta.json" + tmp, stem + ".meta.json")  # meta last: readers wait on it
    return n


class TextDataset(BaseDataset[TextDatasetItem, TextDatasetBatchBeforeSync, TextDatasetBatch]):
    """Fixed-length token items from a memory map (every item has ``sequence_length + 1`` tokens)."""

    def __init__(self, data_prefix: Path, sequence_length: int, seed: int, legacy_dataset: bool = False,
                 load_mmap_index_to_memory: bool = False, load_data_item_mmap_index_to_memory: bool = False,
                 only_full_sequences: bool = False, allow_incomplete_sequences_every_n: int = 0, use_mmap: bool = True,
                 shuffle: bool = True):
        self.use_mmap = use_mmap
        self.data_prefix = Path(data_prefix)
        self.sequence_length = sequence_length
        self.legacy_dataset = legacy_dataset
        self.load_mmap_index_to_memory = load_mmap_index_to_memory
        self.load_data_item_mmap_index_to_memory = load_data_item_mmap_index_to_memory
        self.only_full_sequences = only_full_sequences
        self.allow_incomplete_sequences_every_n = allow_incomplete_sequences_every_n
        if load_mmap_index_to_memory or load_data_item_mmap_index_to_memory:
            assert not legacy_dataset, "cannot load index to memory when using the legacy dataset"
        if legacy_dataset:
            from .legacy_dataset import get_indexed_dataset_

            self.memory_map = get_indexed_dataset_(str(data_prefix), data_impl="mmap", skip_warmup=True)
            assert not only_full_sequences, "full sequences datasets not supported for legacy datasets."
        elif use_mmap:
            self.memory_map = MemoryMapDataset(prefix_path=data_prefix, load_index_to_memory=load_mmap_index_to_memory)
        else:
            self.memory_map = FileDataset(prefix_path=data_prefix, load_index_to_memory=load_mmap_index_to_memory)
        self.seed: Optional[int] = None
        self.data_item_index: Optional[Union[MemoryMapDataset, FileDataset]] = None
        super().__init__(seed=seed, shuffle=shuffle)

    def ident(self) -> str:
        return f"{hashlib.md5(str(self.data_prefix).encode('utf-8')).hexdigest()}-seq-{self.sequence_length}"

    def get_data_index_cache_filename_stem(self, seed: int) -> str:
        stem = str(self.data_prefix) + f"_index_cache_decoder_dataset_seed_{seed}_seq_len_{self.sequence_length}"
        if self.only_full_sequences:
            stem += f"_only_full_sequences_allow_incomplete_sequences_every_n_{self.allow_incomplete_sequences_every_n}"
        return stem

    def get_data_index_cache_filename_bin(self, seed: int) -> str:
        return self.get_data_index_cache_filename_stem(seed) + ".bin"

    def get_data_index_cache_filename_idx(self, seed: int) -> str:
        return self.get_data_index_cache_filename_stem(seed) + ".idx"

    def get_data_index_cache_filename_meta(self, seed: int) -> str:
        return self.get_data_index_cache_filename_stem(seed) + ".meta.json"

    def _doc_sizes(self) -> np.ndarray:
        s = self.memory_map.sizes() if callable(self.memory_map.sizes) else self.memory_map.sizes
        return np.asarray(s, dtype=np.int64)

    def get_data_index_cache_filename_done(self, seed: int) -> str:
        return self.get_data_index_cache_filename_stem(seed) + ".done"

    def compute_data_index(self, seed: int) -> None:
        """Legacy (MMIDIDX) item index: int32 (doc, start, end) triples per item plus a ``.done`` marker
        (reference ``text_dataset.py:125-218``)."""
        if self.seed is not None and self.seed == seed:
            return
        self.seed = seed
        from .legacy_dataset import get_indexed_dataset_
        from .legacy_dataset.indexed_dataset import Index

        stem = self.get_data_index_cache_filename_stem(seed)
        done = self.get_data_index_cache_filename_done(seed)
        if not Path(done).is_file() and _rank() == 0:
            order = np.arange(len(self.memory_map))
            np.random.RandomState(seed=seed).shuffle(order)
            from scaling_amd import _data  # type: ignore[attr-defined]

            flat, pairs = _data.text_index(np.asarray(self.memory_map.sizes, dtype=np.int64), order.astype(np.int64),
                                           int(self.sequence_length), False, 0)
            flat.astype(np.int32).tofile(stem + ".bin")
            Index.write(stem + ".idx", np.int32, pairs.reshape(-1, 2)[:, 1].tolist(), [0])
            Path(done).write_text("True")
        while not (Path(stem + ".bin").is_file() and Path(stem + ".idx").is_file() and Path(done).is_file()):
            time.sleep(0.5)
        self.data_item_index = get_indexed_dataset_(stem, "mmap", True)  # type: ignore[assignment]

    def set_seed(self, seed: int, shuffle: bool = True) -> None:
        if self.legacy_dataset:
            self.compute_data_index(seed)
            return
        if self.seed is not None and self.seed == seed:
            return
        self.seed = seed
        stem = self.get_data_index_cache_filename_stem(seed)
        meta = self.get_data_index_cache_filename_meta(seed)
        if not Path(meta).is_file() and _rank() == 0:
            order = np.arange(len(self.memory_map))
            if shuffle:
                np.random.RandomState(seed=seed).shuffle(order)
            write_text_index(stem, self._doc_sizes(), order, self.sequence_length, self.only_full_sequences,
                             self.allow_incomplete_sequences_every_n)
        waited = 0
        while not (Path(stem + ".bin").is_file() and Path(stem + ".idx").is_file() and Path(meta).is_file()):
            time.sleep(0.5)
            waited += 1
            if waited % 120 == 0:
                print(f"TextDataset waiting on index for seed {seed} on rank {_rank()} ({waited / 120:.1f} min)", flush=True)
        cls = MemoryMapDataset if self.use_mmap else FileDataset
        self.data_item_index = cls(prefix_path=Path(stem), load_index_to_memory=self.load_data_item_mmap_index_to_memory)

    def __len__(self) -> int:
        assert self.data_item_index is not None
        return len(self.data_item_index)

    def __getitem__(self, index: int) -> TextDatasetItem:
        assert self.data_item_index is not None, "data item index not set"
        triples = np.asarray(self.data_item_index[index]).reshape(-1, 3)
        parts = [np.asarray(self.memory_map[int(d)][int(a):int(b)]) for d, a, b in triples]
        tokens = np.concatenate(parts) if len(parts) > 1 else parts[0]
        return TextDatasetItem(token_ids=torch.from_numpy(tokens.astype(np.int64)))

    def collate(self, batch: list[TextDatasetItem]) -> TextDatasetBatchBeforeSync:
        # stays on host: loader workers must not touch the GPU
        return TextDatasetBatchBeforeSync(token_ids=torch.stack([b.token_ids for b in batch]))

    @staticmethod
    def sync_batch_to_model_parallel(topology: Optional[Topology], batch: Optional[TextDatasetBatchBeforeSync]
                                     ) -> TextDatasetBatch:
        if topology is None:
            assert batch is not None
            return TextDatasetBatch(input_token_ids=batch.token_ids[:, :-1], target_token_ids=batch.token_ids[:, 1:])
        if (topology.config.model_parallel_size == 1 and batch is not None and not batch.token_ids.is_cuda
                and topology.device.type == "cuda"):
            return TextDataset._host_derived_batch(batch.token_ids, topology.device)
        if topology.model_parallel_rank == 0:
            assert batch is not None
            tensors: list[Optional[torch.Tensor]] = [batch.token_ids]
        else:
            assert batch is None
            tensors = [None]
        tok = broadcast_data(tensors=tensors, dtype=torch.long, topology=topology)[0]
        return TextDatasetBatch(input_token_ids=tok[:, :-1], target_token_ids=tok[:, 1:])

    @staticmethod
    def _host_derived_batch(token_ids: torch.Tensor, device: torch.device) -> TextDatasetBatch:
        """TP 1 with the batch still on the host: cu_seqlens (plain and -1 padded) and position ids are derived from
        the host copy of the token ids and travel with them as asynchronous pinned copies -- on the device they cost
        ~40 small kernels and a device sync (``torch.nonzero``) per micro-batch, which a small model's host-bound step
        pays in full.  The values are those of ``TextDatasetBatch``'s own derivation (same functions)."""
        from .utils import add_cumulative_seq_lengths_padding, get_cumulative_seq_lengths, get_position_ids

        inp = token_ids[:, :-1]
        b, s = inp.shape
        cu = get_cumulative_seq_lengths(inp)
        host = {"tok": token_ids, "cu": cu, "cu_pad": add_cumulative_seq_lengths_padding(cu, b * (s + 1)),
                "pos": get_position_ids(inp)}
        dev = {k: (v if v.is_pinned() else v.pin_memory()).to(device, non_blocking=True) for k, v in host.items()}
        tok = dev["tok"]
        return TextDatasetBatch(input_token_ids=tok[:, :-1], target_token_ids=tok[:, 1:], position_ids=dev["pos"],
                                cumulative_seq_lengths=dev["cu"], cumulative_seq_lengths_padded=dev["cu_pad"])

    @staticmethod
    def jsonl_to_memory_map(data_file_jsonl: Path, prefix_path_memory_map: Path) -> None:
        """Tokenizes ``{"text": ...}`` lines with the default tokenizer (+ EOS) into a memory map."""
        from ..tokenizer import Tokenizer

        tokenizer = Tokenizer.default()
        with MemoryMapDatasetBuilder(prefix_path=Path(prefix_path_memory_map)) as builder, \
                open(data_file_jsonl, "r", encoding="UTF-8") as f:
            for line in f:
                ids = tokenizer.encode(json.loads(line)["text"]) + [tokenizer.eos_token_id]
                builder.add(np_array=np.array(ids))


class TextBlendedDataset(BaseBlendedDataset[TextDatasetItem, TextDatasetBatchBeforeSync, TextDatasetBatch, TextDataset]):
    pass
