"""Rotary embeddings (reference ``src/scaling/core/nn/rotary.py:142-255``).

Both classes keep the reference call signature ``forward(query, key, query_position_ids,
key_position_ids)`` on ``[sq, b, heads, head_dim]`` tensors, and add ``apply_tokens`` which the
MI355X attention uses directly on token-major ``[T, heads, head_dim]`` views (HIP kernel).
"""
from __future__ import annotations

from typing import Optional

import torch

from ...ops import rope as rope_ops
from .rotary_config import RotaryConfig


class _RotaryBase(torch.nn.Module):
    interleaved = False

    def __init__(self, config: RotaryConfig, device: torch.device, dtype: torch.dtype = torch.float32) -> None:
        super().__init__()
        assert config.dimensions > 1, "RotaryEmbedding cannot use `dim` == 1"
        self.dimensions = config.dimensions
        self.max_seq_length = config.max_seq_length
        cos, sin = rope_ops.rope_tables(
            config.dimensions, config.max_seq_length, config.base, self.interleaved, dtype, device
        )
        self.register_buffer("cos_table", cos, persistent=False)
        self.register_buffer("sin_table", sin, persistent=False)

    def apply_tokens(self, x: torch.Tensor, position_ids: Optional[torch.Tensor], seq_len: int) -> torch.Tensor:
        """x: [T, heads, head_dim] (token-major, T = b*seq_len); position_ids: [b, seq_len] or None."""
        return rope_ops.apply_rope(
            x, self.cos_table, self.sin_table, position_ids, self.dimensions, seq_len, self.interleaved
        )

    def forward(
        self,
        query: torch.Tensor,
        key: torch.Tensor,
        query_position_ids: Optional[torch.Tensor] = None,
        key_position_ids: Optional[torch.Tensor] = None,
    ) -> tuple[torch.Tensor, torch.Tensor]:
        """query/key: [sq, b, heads, hd]; position ids: [sq, b] (reference layout)."""

        def one(x: torch.Tensor, pos: Optional[torch.Tensor]) -> torch.Tensor:
            sq, b, nh, hd = x.shape
            xt = x.transpose(0, 1).reshape(b * sq, nh, hd)
            p = None if pos is None else pos.transpose(0, 1).reshape(-1)
            return self.apply_tokens(xt, p, sq).view(b, sq, nh, hd).transpose(0, 1)

        return one(query, query_position_ids), one(key, key_position_ids)


class RotaryEmbedding(_RotaryBase):
    """NeoX rotate-half convention, optional partial rotation (``dimensions < head_dim``)."""

    interleaved = False


class RotaryEmbeddingComplex(_RotaryBase):
    """LLaMA complex/interleaved convention, computed in fp32."""

    interleaved = True

    def __init__(self, config: RotaryConfig, device: torch.device, dtype: torch.dtype = torch.float32) -> None:
        super().__init__(config, device, torch.float32)
