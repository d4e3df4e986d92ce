"""Embedding head: position-weighted mean pooling (fp32) + projection stack (reference
``model/layers/embedding_head.py``)."""
from __future__ import annotations

from typing import Optional

import torch

from ....core import Topology
from ...context.config import TransformerArchitectureConfig
from .base import TransformerLayerBaseIO, TransformerLayerIO
from .embedding import _device


class TransformerEmbeddingHead(TransformerLayerBaseIO):
    def __init__(self, architecture_config: TransformerArchitectureConfig, topology: Optional[Topology] = None):
        super().__init__()
        assert architecture_config.embedding_head_config is not None, "EmbeddingHead needs embedding_head_config"
        self.architecture_config = architecture_config
        self.topology = topology
        self.embedding_head_config = architecture_config.embedding_head_config
        n_in = architecture_config.hidden_size
        for i, n_out in enumerate(self.embedding_head_config.proj_layers):
            setattr(self, f"embedding_head_proj_{self.embedding_head_config.name}_{i}",
                    torch.nn.Linear(n_in, n_out, bias=False, device=_device(topology), dtype=architecture_config.precision.dtype))
            n_in = n_out

    def forward(self, x: TransformerLayerIO) -> TransformerLayerIO:
        assert x.loss_weights is not None, "did not receive loss_weights for masking"
        act = self.weighted_mean_pooling(x.activations, x.loss_weights)
        if self.embedding_head_config.proj_layers:
            act = self.apply_embedding_head_proj(act)
        return x.derive(act, attention_scores_manipulation=None)

    @staticmethod
    def weighted_mean_pooling(embeddings: torch.Tensor, loss_weights: torch.Tensor) -> torch.Tensor:
        in_dtype = embeddings.dtype
        e = embeddings.float()
        pos = torch.arange(1, e.shape[1] + 1, dtype=e.dtype, device=e.device).view(1, -1, 1)
        w = loss_weights.to(e.dtype).unsqueeze(-1) * pos
        num = (e * w).sum(dim=1)
        den = w.expand_as(e).sum(dim=1)
        if float(den.sum()) == 0.0:
            return torch.zeros_like(num).to(in_dtype)
        return (num / den).to(in_dtype)

    def apply_embedding_head_proj(self, embeddings: torch.Tensor) -> torch.Tensor:
        for i, _ in enumerate(self.embedding_head_config.proj_layers):
            if i > 0:
                embeddings = torch.nn.functional.gelu(embeddings)
            embeddings = getattr(self, f"embedding_head_proj_{self.embedding_head_config.name}_{i}")(embeddings)
        return embeddings
