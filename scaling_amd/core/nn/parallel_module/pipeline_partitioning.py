"""Assignment of layers to pipeline stages.

``uniform`` spreads the remainder over the first stages (reference ``pipeline_partitioning.py:38``);
``balanced`` minimises the largest per-stage parameter count over contiguous partitions (exact
binary search on the bottleneck + greedy packing; layers are built one at a time on CPU to count).
"""
from __future__ import annotations

from typing import NamedTuple, Optional, Sequence

import numpy as np


class PipePartitionCoordinates(NamedTuple):
    start: int
    end: int

    @property
    def length(self) -> int:
        return self.end - self.start


def pipe_partition_from_indices(partition_array: Sequence[int], num_layers: Optional[int] = None) -> list[PipePartitionCoordinates]:
    if num_layers is not None and partition_array[-1] != num_layers:
        raise ValueError(
            f"Last entry of partition_array needs to match num_layers; got partition_array={partition_array}, "
            f"num_layers={num_layers}."
        )
    return [PipePartitionCoordinates(int(s), int(e)) for s, e in zip(partition_array[:-1], partition_array[1:])]


def pipe_partition_uniform(item_count: int, partition_count: int) -> list[PipePartitionCoordinates]:
    assert item_count >= partition_count, f"cannot partition {item_count} layers on {partition_count} pipe parallel stages"
    base, rest = divmod(item_count, partition_count)
    bounds = [0]
    for p in range(partition_count):
        bounds.append(bounds[-1] + base + (1 if p < rest else 0))
    return pipe_partition_from_indices(bounds)


def _pack(weights: Sequence[int], parts: int, cap: int) -> Optional[list[int]]:
    """Greedy contiguous packing with at most `cap` per part (each part non-empty); None if infeasible."""
    n = len(weights)
    bounds, cur, start = [0], 0, 0
    for i, w in enumerate(weights):
        if w > cap:
            return None
        remaining_parts = parts - (len(bounds) - 1)
        remaining_items = n - i
        if (cur + w > cap or remaining_items < remaining_parts) and i > start:
            bounds.append(i)
            start, cur = i, 0
        cur += w
    bounds.append(n)
    if len(bounds) - 1 > parts:
        return None
    while len(bounds) - 1 < parts:  # split the last multi-layer part to keep every stage non-empty
        for j in range(len(bounds) - 1, 0, -1):
            if bounds[j] - bounds[j - 1] > 1:
                bounds.insert(j, bounds[j] - 1)
                break
        else:
            return None
    return bounds


def partition_balanced_weights(weights: Sequence[int], partition_count: int) -> list[PipePartitionCoordinates]:
    assert len(weights) >= partition_count
    lo, hi = max(weights) if len(weights) else 0, int(sum(weights))
    best = _pack(weights, partition_count, hi)
    while lo < hi:
        mid = (lo + hi) // 2
        b = _pack(weights, partition_count, mid)
        if b is not None:
            hi, best = mid, b
        else:
            lo = mid + 1
    b = _pack(weights, partition_count, lo)
    best = b if b is not None else best
    assert best is not None
    return pipe_partition_from_indices(best)


def _count_layer_params(layer_specs: list) -> list[int]:
    import torch

    counts = []
    for spec in layer_specs:
        kwargs = dict(spec.kwargs)
        layer = spec.module_class(**kwargs)
        counts.append(sum(p.numel() for p in layer.parameters() if p.requires_grad))
        del layer
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    return counts


def pipe_partition_balanced(layer_specs: list, partition_count: int, eps: float = 1e-3) -> list[PipePartitionCoordinates]:
    return partition_balanced_weights(_count_layer_params(layer_specs), partition_count)


__all__ = [
    "PipePartitionCoordinates",
    "np",
    "partition_balanced_weights",
    "pipe_partition_balanced",
    "pipe_partition_from_indices",
    "pipe_partition_uniform",
]
