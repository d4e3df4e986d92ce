"""Layer IO of the transformer pipeline (reference ``model/layers/base.py:12-123``)."""
from __future__ import annotations

from typing import Any, Optional

import torch

from ....core import BaseLayer, BaseLayerIO
from ...data.inference_settings import InferenceSettings


class TransformerLayerIO(BaseLayerIO):
    _FIELDS = ("activations", "position_ids", "cumulative_seq_lengths", "cumulative_seq_lengths_padded",
               "loss_weights", "inference_settings", "embeddings", "embeddings_head", "attention_scores_manipulation",
               "residual_branch")

    @staticmethod
    def field_names() -> list[str]:
        return list(TransformerLayerIO._FIELDS)

    def as_tuple(self) -> tuple[Any, ...]:
        names = [n for n in self._FIELDS if getattr(self, n) is not None]
        return tuple([getattr(self, n) for n in names] + [names])

    @classmethod
    def from_tuple(cls, d: tuple[Any, ...]) -> "TransformerLayerIO":
        names, values = d[-1], d[:-1]
        assert len(names) == len(values)
        return cls(**dict(zip(names, values)))

    def __init__(
        self,
        activations: torch.Tensor,
        position_ids: torch.Tensor,
        cumulative_seq_lengths_padded: torch.Tensor,
        cumulative_seq_lengths: Optional[torch.Tensor] = None,
        loss_weights: Optional[torch.Tensor] = None,
        inference_settings: Optional[InferenceSettings] = None,
        embeddings: Optional[torch.Tensor] = None,
        embeddings_head: Optional[torch.Tensor] = None,
        attention_scores_manipulation: Optional[torch.Tensor] = None,
        residual_branch: Optional[torch.Tensor] = None,
    ) -> None:
        self.activations = activations
        # a transformer layer may hand over its hidden state as (activations, residual_branch) with the MLP's residual
        # add still pending: the next layer's input norm does that add inside its kernel (one HBM pass and one launch
        # less per layer); every consumer takes ``hidden()`` or the add-norm
        self.residual_branch = residual_branch
        self.position_ids = position_ids
        self.cumulative_seq_lengths = cumulative_seq_lengths
        self.cumulative_seq_lengths_padded = cumulative_seq_lengths_padded
        self.loss_weights = loss_weights
        self.inference_settings = inference_settings
        self.embeddings = embeddings
        self.embeddings_head = embeddings_head
        self.attention_scores_manipulation = attention_scores_manipulation
        # (vocab_start, tp_group, tp_size) when `activations` are vocab-sharded logits (never communicated)
        self.vocab_parallel: Optional[tuple[int, Any, int]] = None
        self.max_seq_length: Optional[int] = None

    def hidden(self) -> torch.Tensor:
        """The hidden state with a pending residual add applied."""
        if self.residual_branch is None:
            return self.activations
        return self.activations + self.residual_branch

    def derive(self, activations: torch.Tensor, **overrides: Any) -> "TransformerLayerIO":
        kw = {n: getattr(self, n) for n in self._FIELDS}
        kw["residual_branch"] = None  # a pending add belongs to the activations it came with
        kw.update(activations=activations, **overrides)
        out = TransformerLayerIO(**kw)
        out.max_seq_length = self.max_seq_length
        return out


class TransformerLayerBaseIO(BaseLayer[TransformerLayerIO, TransformerLayerIO, TransformerLayerIO]):
    @staticmethod
    def input_to_tuple(input: TransformerLayerIO) -> tuple[Any, ...]:
        return input.as_tuple()

    @staticmethod
    def tuple_to_input(d: tuple[Any, ...]) -> TransformerLayerIO:
        return TransformerLayerIO.from_tuple(d)

    @staticmethod
    def output_to_tuple(output: TransformerLayerIO) -> tuple[Any, ...]:
        return output.as_tuple()

    @staticmethod
    def tuple_to_last_stage_activation(d: tuple[Any, ...]) -> TransformerLayerIO:
        return TransformerLayerIO.from_tuple(d)
