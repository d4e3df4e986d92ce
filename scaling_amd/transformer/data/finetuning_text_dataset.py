"""Prompt/completion finetuning data (reference ``transformer/data/finetuning_text_dataset.py``).

Sources: a JSON list of ``{"prompt": str | [str | "*.jpg", ...], "completion": str}`` or a memory map
whose documents are ``[len(prompt), *prompt_ids, *completion_ids]`` (``convert_jsonl``).  Every item is
padded with EOS to ``sequence_length + 1``; the loss covers the completion plus one EOS.
"""
from __future__ import annotations

import hashlib
import json
import random
from pathlib import Path
from typing import Any, Optional, Union

import numpy as np
import torch

from ...core import BaseBlendedDataset, BaseDataset, BaseDatasetItem, MemoryMapDataset, MemoryMapDatasetBuilder, Topology
from ...core import broadcast_data
from ..tokenizer import Tokenizer
from .text_dataset_batch import TextDatasetBatch
from .utils import get_cumulative_seq_lengths

IMAGE_ENCODER_TOKEN_COUNTS = 144
IMAGE_SIZE = (384, 384)

_TRANSFORM = None


def image_transform() -> Any:
    global _TRANSFORM
    if _TRANSFORM is None:
        from ..model.image_encoder import clip_transform

        _TRANSFORM = clip_transform(IMAGE_SIZE)
    return _TRANSFORM


def load_image(path: Path) -> torch.Tensor:
    from PIL import Image

    return image_transform()(Image.open(str(path)))


class FinetuningTextDatasetItem(BaseDatasetItem):
    def __init__(self, input_token_ids: torch.Tensor, target_token_ids: torch.Tensor, cumulative_seq_lengths: torch.Tensor,
                 position_ids: torch.Tensor, loss_weights: torch.Tensor, input_images: Optional[list[torch.Tensor]] = None,
                 input_image_locations: Optional[list[tuple[int, int]]] = None):
        super().__init__()
        self.input_token_ids = input_token_ids
        self.target_token_ids = target_token_ids
        self.cumulative_seq_lengths = cumulative_seq_lengths
        self.position_ids = position_ids
        self.loss_weights = loss_weights
        self.input_images = input_images
        self.input_image_locations = input_image_locations


def _shift_locations(locs: Optional[list[tuple[int, int]]], n: int) -> Optional[list[tuple[int, int]]]:
    return None if locs is None else [(a + n, b + n) for a, b in locs]


def collate_finetuning(batch: list[FinetuningTextDatasetItem]) -> TextDatasetBatch:
    """Stack items (host tensors); images are flattened with (item, start, end) locations."""
    stack = lambda name: torch.stack([getattr(b, name) for b in batch])  # noqa: E731
    input_token_ids = stack("input_token_ids")
    images, locs = [], []
    for i, b in enumerate(batch):
        for img, (s, e) in zip(b.input_images or [], b.input_image_locations or []):
            images.append(img)
            locs.append([i, s, e])
    return TextDatasetBatch(
        input_token_ids=input_token_ids,
        target_token_ids=stack("target_token_ids"),
        cumulative_seq_lengths=get_cumulative_seq_lengths(input_token_ids, reset_attention_mask=False),
        position_ids=stack("position_ids"),
        loss_weights=stack("loss_weights"),
        input_images=torch.stack(images) if images else None,
        input_image_locations=torch.tensor(locs, dtype=torch.long) if locs else None,
    )


def sync_finetuning_batch(topology: Optional[Topology], batch: Optional[TextDatasetBatch]) -> TextDatasetBatch:
    """Broadcast a finetuning batch from TP rank 0: one int64 and one fp32 flat broadcast."""
    if topology is None:
        assert batch is not None
        return batch
    if topology.model_parallel_rank == 0:
        assert batch is not None
        batch.contiguous_()
        assert batch.cumulative_seq_lengths_padded is not None
        longs: list[Optional[torch.Tensor]] = [
            batch.input_token_ids, batch.target_token_ids, batch.cumulative_seq_lengths_padded.to(torch.long),
            batch.position_ids,
            batch.input_image_locations if batch.input_image_locations is not None else torch.tensor([-1], dtype=torch.long),
        ]
        floats: list[Optional[torch.Tensor]] = [
            batch.loss_weights,
            batch.input_images if batch.input_images is not None else torch.tensor([-1.0]),
        ]
    else:
        assert batch is None
        longs, floats = [None] * 5, [None] * 2
    L = broadcast_data(tensors=longs, dtype=torch.long, topology=topology)
    F = broadcast_data(tensors=floats, dtype=torch.float32, topology=topology)
    has_images = L[4].dim() == 2  # the "no images" marker is the 1-D tensor [-1]
    return TextDatasetBatch(
        input_token_ids=L[0], target_token_ids=L[1], cumulative_seq_lengths_padded=L[2].to(torch.int32),
        position_ids=L[3], loss_weights=F[0],
        input_images=F[1] if has_images else None, input_image_locations=L[4] if has_images else None,
    )


class FinetuningTextDataset(BaseDataset[FinetuningTextDatasetItem, TextDatasetBatch, TextDatasetBatch]):
    def __init__(self, data_prefix: Path, sequence_length: int, seed: int, softprompt_n_tokens: int, tokenizer: Tokenizer,
                 tokenizer_no_prefix_space: Tokenizer, memory_map_dataset: bool = False, shuffle: bool = True):
        self.data_prefix = Path(data_prefix)
        self.data_prefix_parent = self.data_prefix.parent
        self.sequence_length = sequence_length
        self.softprompt_n_tokens = softprompt_n_tokens
        self.tokenizer = tokenizer
        self.tokenizer_no_prefix_space = tokenizer_no_prefix_space
        self.memory_map_dataset = memory_map_dataset
        self.dataset: Optional[MemoryMapDataset] = None
        if memory_map_dataset:
            self.dataset = MemoryMapDataset(prefix_path=self.data_prefix)
            self.data: list[Any] = list(range(len(self.dataset)))
        else:
            with open(self.data_prefix, "r", encoding="UTF-8") as f:
                self.data = json.load(f)
        self.seed: Optional[int] = None
        super().__init__(seed=seed, shuffle=shuffle)

    def ident(self) -> str:
        h = hashlib.md5(str(self.data_prefix).encode("utf-8"))
        if not self.memory_map_dataset:
            for t in (self.tokenizer, self.tokenizer_no_prefix_space):
                h.update(json.dumps(t.tokenizer.get_vocab(), sort_keys=True, default=str).encode("utf-8"))
        return f"{h.hexdigest()}-seq-{self.sequence_length}"

    def set_seed(self, seed: int, shuffle: bool = True) -> None:
        if self.seed is not None and self.seed == seed:
            return
        random.seed(seed)
        if shuffle:
            random.shuffle(self.data)
        self.seed = seed

    def __len__(self) -> int:
        return len(self.data)

    def get_memory_map_token_ids(self, index: int) -> tuple[list[int], list[int]]:
        assert self.dataset is not None
        ids = self.dataset[self.data[index]].tolist()
        n = ids[0]
        return ids[1 : n + 1], ids[n + 1 :]

    def get_json_token_ids(self, index: int) -> tuple[list[int], list[int], Optional[list[torch.Tensor]],
                                                        Optional[list[tuple[int, int]]]]:
        item = self.data[index]
        prompt = item["prompt"]
        images: Optional[list[torch.Tensor]] = None
        locs: Optional[list[tuple[int, int]]] = None
        if isinstance(prompt, list):
            ids: list[int] = []
            images, locs = [], []
            for i, part in enumerate(prompt):
                assert isinstance(part, str)
                img_path = self.data_prefix_parent / part
                is_image = False
                if part.endswith(".jpg"):
                    try:
                        is_image = img_path.is_file()
                    except OSError:  # e.g. "File name too long": it is text
                        is_image = False
                if is_image:
                    images.append(load_image(img_path))
                    locs.append((len(ids), len(ids) + IMAGE_ENCODER_TOKEN_COUNTS))
                    ids.extend([self.tokenizer.eos_token_id] * IMAGE_ENCODER_TOKEN_COUNTS)
                else:
                    ids.extend((self.tokenizer if i == 0 else self.tokenizer_no_prefix_space).encode(part))
        else:
            assert isinstance(prompt, str)
            ids = self.tokenizer.encode(prompt)
        return ids, self.tokenizer.encode(item["completion"]), images, locs

    def __getitem__(self, index: int) -> FinetuningTextDatasetItem:
        eos = self.tokenizer.eos_token_id
        if self.memory_map_dataset:
            prompt, completion = self.get_memory_map_token_ids(index)
            images, locs = None, None
        else:
            prompt, completion, images, locs = self.get_json_token_ids(index)
        if self.softprompt_n_tokens > 0:
            prompt = [0] * self.softprompt_n_tokens + prompt
            locs = _shift_locations(locs, self.softprompt_n_tokens)
        S = self.sequence_length
        pad = S - len(prompt) - len(completion) + 1
        ids = (prompt + completion + [eos] * pad)[: S + 1]
        loss_weights = torch.ones(S, dtype=torch.float)
        loss_weights[: len(prompt) - 1] = 0
        if pad - 1 > 0:  # keep the first EOS as a target, mask the rest of the padding
            loss_weights[-(pad - 1):] = 0
        return FinetuningTextDatasetItem(
            input_token_ids=torch.tensor(ids[:-1], dtype=torch.long),
            target_token_ids=torch.tensor(ids[1:], dtype=torch.long),
            cumulative_seq_lengths=torch.tensor([0, S], dtype=torch.int32),
            position_ids=torch.arange(0, S),
            loss_weights=loss_weights,
            input_images=images,
            input_image_locations=locs,
        )

    def collate(self, batch: list[FinetuningTextDatasetItem]) -> TextDatasetBatch:
        return collate_finetuning(batch)

    @staticmethod
    def sync_batch_to_model_parallel(topology: Optional[Topology], batch: Optional[TextDatasetBatch]) -> TextDatasetBatch:
        return sync_finetuning_batch(topology, batch)

    @staticmethod
    def convert_jsonl(jsonl_file: Union[str, Path], tokenizer: Tokenizer, tokenizer_no_prefix_space: Tokenizer,
                      out_prefix_path: Union[str, Path]) -> None:
        with MemoryMapDatasetBuilder(prefix_path=Path(out_prefix_path)) as builder, \
                open(jsonl_file, "r", encoding="UTF-8") as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                d = json.loads(line)
                p = tokenizer.encode(d["prompt"])
                c = tokenizer_no_prefix_space.encode(d["completion"])
                builder.add(np_array=np.array([len(p)] + p + c))


class FinetuningTextBlendedDataset(
    BaseBlendedDataset[FinetuningTextDatasetItem, TextDatasetBatch, TextDatasetBatch, FinetuningTextDataset]
):
    pass
