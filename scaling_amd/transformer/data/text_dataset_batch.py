"""Text batches (reference ``data/text_dataset_batch.py:29-140``): derived cu_seqlens (+ -1 padded
copy of fixed length ``b*(s+1)`` for pipeline p2p), position ids, loss weights."""
from __future__ import annotations

from typing import Any, Optional

import torch

from ...core import BaseDatasetBatch
from .inference_settings import InferenceSettings
from .utils import (
    add_cumulative_seq_lengths_padding,
    get_cumulative_seq_lengths,
    get_position_ids,
    remove_cumulative_seq_lengths_padding,
)


class TextDatasetBatchBeforeSync(BaseDatasetBatch):
    def __init__(self, token_ids: torch.Tensor):
        self.token_ids = token_ids

    def only_inputs(self) -> "TextDatasetBatchBeforeSync":
        return self

    def only_targets(self) -> "TextDatasetBatchBeforeSync":
        return self


class TextDatasetBatch(BaseDatasetBatch):
    _FIELDS = ("input_token_ids", "input_images", "input_image_locations", "target_token_ids", "position_ids",
               "cumulative_seq_lengths", "cumulative_seq_lengths_padded", "loss_weights", "inference_settings",
               "embeddings")

    @staticmethod
    def field_names() -> list[str]:
        return list(TextDatasetBatch._FIELDS)

    def as_tuple(self) -> tuple[Any, ...]:
        names = [n for n in self._FIELDS if getattr(self, n) is not None]
        return tuple([getattr(self, n) for n in names] + [names])

    @classmethod
    def from_tuple(cls, d: tuple[Any, ...]) -> "TextDatasetBatch":
        names, values = d[-1], d[:-1]
        assert len(names) == len(values)
        return cls(**dict(zip(names, values)))

    def __init__(
        self,
        input_token_ids: Optional[torch.Tensor] = None,
        input_images: Optional[torch.Tensor] = None,
        input_image_locations: Optional[torch.Tensor] = None,
        target_token_ids: Optional[torch.Tensor] = None,
        position_ids: Optional[torch.Tensor] = None,
        cumulative_seq_lengths: Optional[torch.Tensor] = None,
        cumulative_seq_lengths_padded: Optional[torch.Tensor] = None,
        loss_weights: Optional[torch.Tensor] = None,
        inference_settings: Optional[InferenceSettings] = None,
        embeddings: Optional[torch.Tensor] = None,
    ) -> None:
        self.input_token_ids = input_token_ids
        self.input_images = input_images
        self.input_image_locations = input_image_locations
        self.target_token_ids = target_token_ids
        self.position_ids = position_ids
        self.cumulative_seq_lengths = cumulative_seq_lengths
        self.cumulative_seq_lengths_padded = cumulative_seq_lengths_padded
        self.loss_weights = loss_weights
        self.inference_settings = inference_settings
        self.embeddings = embeddings
        if input_token_ids is not None:
            if self.cumulative_seq_lengths is None:
                self.cumulative_seq_lengths = (
                    remove_cumulative_seq_lengths_padding(self.cumulative_seq_lengths_padded)
                    if self.cumulative_seq_lengths_padded is not None
                    else get_cumulative_seq_lengths(input_token_ids)
                )
            if self.cumulative_seq_lengths_padded is None:
                b, s = input_token_ids.shape
                self.cumulative_seq_lengths_padded = add_cumulative_seq_lengths_padding(self.cumulative_seq_lengths, b * (s + 1))
            if self.position_ids is None:
                self.position_ids = get_position_ids(input_token_ids)
            if self.loss_weights is None:
                self.loss_weights = torch.ones_like(input_token_ids, dtype=torch.float).contiguous()

    def contiguous_(self) -> "TextDatasetBatch":
        for n in self._FIELDS:
            v = getattr(self, n)
            if isinstance(v, torch.Tensor):
                setattr(self, n, v.contiguous())
        return self

    def only_inputs(self) -> "TextDatasetBatch":
        return TextDatasetBatch(input_token_ids=self.input_token_ids, input_images=self.input_images,
                                input_image_locations=self.input_image_locations, position_ids=self.position_ids,
                                cumulative_seq_lengths=self.cumulative_seq_lengths)

    def only_targets(self) -> "TextDatasetBatch":
        return TextDatasetBatch(target_token_ids=self.target_token_ids, loss_weights=self.loss_weights)
