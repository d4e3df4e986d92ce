"""Token bookkeeping: cu_seqlens (EOD resets), -1-padded cu_seqlens for fixed-shape p2p, position ids.

Semantics of reference ``transformer/data/utils.py:4-108`` (EOD token id 0; the last token of every
row closes a segment).  ``get_position_ids`` is vectorised (no per-batch Python loop).
"""
from __future__ import annotations

import torch


def add_cumulative_seq_lengths_padding(cumulative_seq_lengths: torch.Tensor, pad_to: int, padding_value: int = -1) -> torch.Tensor:
    assert pad_to >= len(cumulative_seq_lengths)
    pad = torch.full((pad_to - len(cumulative_seq_lengths),), padding_value, dtype=torch.int32,
                     device=cumulative_seq_lengths.device)
    return torch.cat((cumulative_seq_lengths.to(torch.int32), pad))


def remove_cumulative_seq_lengths_padding(cumulative_seq_lengths: torch.Tensor, padding_value: int = -1) -> torch.Tensor:
    return cumulative_seq_lengths[cumulative_seq_lengths != padding_value]


def _segment_ends(input_token_ids: torch.Tensor, eod_token: int) -> torch.Tensor:
    b, s = input_token_ids.shape
    last = torch.zeros_like(input_token_ids, dtype=torch.bool)
    last[:, -1] = True
    return (input_token_ids == eod_token) | last


def get_cumulative_seq_lengths(input_token_ids: torch.Tensor, reset_attention_mask: bool = True, eod_token: int = 0) -> torch.Tensor:
    b, s = input_token_ids.shape
    if not reset_attention_mask:
        return torch.arange(0, b * s + 1, s, dtype=torch.int32, device=input_token_ids.device)
    ends = torch.nonzero(_segment_ends(input_token_ids, eod_token).reshape(-1)).reshape(-1) + 1
    zero = torch.zeros(1, dtype=torch.int32, device=input_token_ids.device)
    return torch.cat([zero, ends.to(torch.int32)])


def get_position_ids(input_token_ids: torch.Tensor, reset_position_ids: bool = True, eod_token: int = 0) -> torch.Tensor:
    b, s = input_token_ids.shape
    ar = torch.arange(s, device=input_token_ids.device).unsqueeze(0).expand(b, s)
    if not reset_position_ids:
        return ar.clone()
    ends = _segment_ends(input_token_ids, eod_token)
    # start of the segment containing position j = (index of previous segment end) + 1
    prev_end = torch.where(ends, ar, torch.full_like(ar, -1))
    prev_end = torch.cat([torch.full((b, 1), -1, device=ar.device, dtype=ar.dtype), prev_end[:, :-1]], dim=1)
    seg_start = torch.cummax(prev_end, dim=1).values + 1
    return (ar - seg_start).to(input_token_ids.dtype)
