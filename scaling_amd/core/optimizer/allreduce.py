"""Small collective helpers (reference ``optimizer/allreduce.py``)."""
from __future__ import annotations

from typing import Any

import torch
import torch.distributed as dist


def allreduce_tensor_in_float32(tensor: torch.Tensor, process_group: Any) -> None:
    """In-place sum over `process_group` accumulated in fp32 (tied grads, TP-constant grads)."""
    if tensor.dtype == torch.float32:
        dist.all_reduce(tensor, group=process_group)
        return
    t = tensor.float()
    dist.all_reduce(t, group=process_group)
    tensor.copy_(t)


def allreduce_no_retain(bucket: list[torch.Tensor], data_parallel_group: Any, data_parallel_size: int,
                        numel_per_bucket: int = 500_000_000) -> None:
    """Average a list of tensors over data parallel in fp32, packed into flat buckets."""
    cur: list[torch.Tensor] = []
    n = 0

    def flush() -> None:
        if not cur:
            return
        flat = torch.cat([t.reshape(-1).float() for t in cur])
        flat.div_(data_parallel_size)
        dist.all_reduce(flat, group=data_parallel_group)
        off = 0
        for t in cur:
            t.copy_(flat[off : off + t.numel()].view_as(t))
            off += t.numel()

    for t in bucket:
        cur.append(t)
        n += t.numel()
        if n >= numel_per_bucket:
            flush()
            cur, n = [], 0
    flush()
