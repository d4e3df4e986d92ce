"""Tensor-parallel batch sync (reference ``core/data/broadcast_data.py:14-165``).

mp-rank 0 packs the shapes (max 8 dims, -1 padded), broadcasts them, then broadcasts one flat
buffer of same-dtype tensors (bool sent as int8).  Works on RCCL and gloo (device = topology device).
"""
from __future__ import annotations

from typing import Any, Optional

import torch
import torch.distributed as dist

_MAX_DATA_DIM = 8


def _build_tensor_sizes(tensors: list[Optional[torch.Tensor]], model_parallel_rank: int) -> list[int]:
    sizes = [-1] * _MAX_DATA_DIM * len(tensors)
    if model_parallel_rank != 0:
        return sizes
    for i, t in enumerate(tensors):
        assert t is not None
        assert t.dim() <= _MAX_DATA_DIM, "you should increase MAX_DATA_DIM"
        for j, s in enumerate(t.size()):
            assert s > 0, "cannot communicate tensor of size 0"
            sizes[i * _MAX_DATA_DIM + j] = s
    return sizes


def _unpack_sizes(flat: list[int]) -> tuple[list[list[int]], list[int]]:
    sizes, numels = [], []
    for i in range(len(flat) // _MAX_DATA_DIM):
        size = []
        for s in flat[i * _MAX_DATA_DIM : (i + 1) * _MAX_DATA_DIM]:
            if s <= 0:
                break
            size.append(s)
        n = 1
        for s in size:
            n *= s
        sizes.append(size)
        numels.append(n)
    return sizes, numels


def _src(topology: Any) -> int:
    return dist.get_global_rank(topology.model_parallel_group, 0)


def sync_sizes(tensors: list[Optional[torch.Tensor]], topology: Any) -> tuple[list[list[int]], list[int]]:
    t = torch.tensor(_build_tensor_sizes(tensors, topology.model_parallel_rank), dtype=torch.long, device=topology.device)
    dist.broadcast(t, _src(topology), group=topology.model_parallel_group)
    return _unpack_sizes(t.cpu().tolist())


def broadcast_data(tensors: list[Optional[torch.Tensor]], dtype: torch.dtype, topology: Any) -> list[torch.Tensor]:
    if topology.config.model_parallel_size == 1:
        # nothing to broadcast: one async H2D copy per tensor (pinned when coming from the loader)
        out = []
        for t in tensors:
            assert t is not None and t.dtype == dtype, f"broadcast_data expects tensors of dtype {dtype}"
            out.append(t.to(topology.device, non_blocking=True))
        return out
    sizes, numels = sync_sizes(tensors, topology)
    if topology.model_parallel_rank == 0:
        for t in tensors:
            assert t is not None and t.dtype == dtype, (
                f"broadcast_data requires a list of tensors of the same dtype; expected {dtype}"
            )
        flat = torch.cat([t.contiguous().view(-1) for t in tensors]).to(topology.device)  # type: ignore[union-attr]
    else:
        flat = torch.empty(sum(numels), dtype=dtype, device=topology.device)
    is_bool = flat.dtype == torch.bool
    if is_bool:
        flat = flat.to(torch.int8)
    dist.broadcast(flat, _src(topology), group=topology.model_parallel_group)
    if is_bool:
        flat = flat.to(torch.bool)
    out, off = [], 0
    for size, n in zip(sizes, numels):
        out.append(flat.narrow(0, off, n).view(size))
        off += n
    return out
