"""Chat finetuning data (reference ``transformer/data/finetuning_chat_dataset.py``): each JSONL line is a
list of ``{"type": "text" | "image", "content": ..., "has_loss": bool}`` elements.  Loss is taken on
tokens of elements with ``has_loss``; sequences are EOS-padded/truncated to ``sequence_length``.
No EOS is appended automatically."""
from __future__ import annotations

import hashlib
import json
import random
from pathlib import Path
from typing import Any, Optional

import torch

from ...core import BaseBlendedDataset, BaseDataset, Topology
from ..tokenizer import Tokenizer
from .finetuning_text_dataset import (
    IMAGE_ENCODER_TOKEN_COUNTS,
    FinetuningTextDatasetItem,
    _shift_locations,
    collate_finetuning,
    load_image,
    sync_finetuning_batch,
)
from .text_dataset_batch import TextDatasetBatch


class FinetuningChatDataset(BaseDataset[FinetuningTextDatasetItem, TextDatasetBatch, TextDatasetBatch]):
    def __init__(self, data_path: Path, sequence_length: int, seed: int, softprompt_n_tokens: int, tokenizer: Tokenizer,
                 tokenizer_no_prefix_space: Tokenizer, shuffle: bool = True):
        self.data_path = Path(data_path)
        self.data_path_parent = self.data_path.parent
        self.sequence_length = sequence_length
        self.softprompt_n_tokens = softprompt_n_tokens
        self.tokenizer = tokenizer
        self.tokenizer_no_prefix_space = tokenizer_no_prefix_space
        with open(self.data_path, "r", encoding="UTF-8") as f:
            self.data_jsonl: list[list[dict[str, Any]]] = [json.loads(s) for s in f.read().split("\n") if s != ""]
        self.data: list[dict[str, Any]] = []
        self.seed: Optional[int] = None
        self.load_data()
        super().__init__(seed=seed, shuffle=shuffle)

    def load_data(self) -> None:
        eos = self.tokenizer.eos_token_id
        warned = False
        for conv in self.data_jsonl:
            ids: list[int] = []
            mask: list[int] = []
            img_paths: Optional[list[Path]] = None
            locs: Optional[list[tuple[int, int]]] = None
            first_text = True
            for el in conv:
                kind, content, has_loss = el["type"], el["content"], bool(el.get("has_loss", False))
                if kind == "text":
                    tok = (self.tokenizer if first_text else self.tokenizer_no_prefix_space).encode(content)
                    ids.extend(tok)
                    mask.extend([int(has_loss)] * len(tok))
                    first_text = False
                elif kind == "image":
                    img_paths = (img_paths or []) + [self.data_path / content]
                    locs = (locs or []) + [(len(ids), len(ids) + IMAGE_ENCODER_TOKEN_COUNTS)]
                    ids.extend([eos] * IMAGE_ENCODER_TOKEN_COUNTS)
                else:
                    raise NotImplementedError(f"Content type {kind} is not supported")
            if eos not in ids and not warned:
                warned = True
                print("WARNING: No EOS Token detected. The 'finetuning_chat_dataset' does not add an EOS token; "
                      "add it to your 'data.jsonl' yourself.")
            self.data.append({"input_token_list": ids[:-1], "target_token_list": ids[1:], "loss_mask_list": mask[1:],
                              "prompt_images_path": img_paths, "prompt_image_locations": locs})

    def ident(self) -> str:
        h = hashlib.md5(str(self.data_path).encode("utf-8"))
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

    def __getitem__(self, index: int) -> FinetuningTextDatasetItem:
        eos = self.tokenizer.eos_token_id
        d = self.data[index]
        inp, tgt, mask = d["input_token_list"], d["target_token_list"], d["loss_mask_list"]
        locs = d["prompt_image_locations"]
        n = self.softprompt_n_tokens
        if n > 0:
            inp, tgt, mask = [0] * n + inp, [0] * n + tgt, [0] * n + mask
            locs = _shift_locations(locs, n)
        S = self.sequence_length
        pad = S - len(inp)
        inp = (inp + [eos] * pad)[:S]
        tgt = (tgt + [eos] * pad)[:S]
        mask = (mask + [0] * pad)[:S]
        images = None
        if d["prompt_images_path"] is not None:
            images = [load_image(self.data_path_parent / p) for p in d["prompt_images_path"]]
        return FinetuningTextDatasetItem(
            input_token_ids=torch.tensor(inp, dtype=torch.long), target_token_ids=torch.tensor(tgt, dtype=torch.long),
            cumulative_seq_lengths=torch.tensor([0, S], dtype=torch.int32), position_ids=torch.arange(0, S),
            loss_weights=torch.tensor(mask, dtype=torch.float32), input_images=images, input_image_locations=locs,
        )

    def collate(self, batch: list[FinetuningTextDatasetItem]) -> TextDatasetBatch:
        return collate_finetuning(batch)

    @staticmethod
    def sync_batch_to_model_parallel(topology: Optional[Topology], batch: Optional[TextDatasetBatch]) -> TextDatasetBatch:
        return sync_finetuning_batch(topology, batch)


class FinetuningChatBlendedDataset(
    BaseBlendedDataset[FinetuningTextDatasetItem, TextDatasetBatch, TextDatasetBatch, FinetuningChatDataset]
):
    pass
