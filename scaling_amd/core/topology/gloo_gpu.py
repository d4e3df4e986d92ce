"""Stream-ordered collectives for the 1-GPU rehearsal mode (``TopologyConfig.gloo_on_gpu``).

In the rehearsal several ranks share one MI355X and gloo stands in for RCCL.  gloo is not a HIP-stream-aware
backend: handed GPU tensors, it moves their bytes from its own worker threads, not in the order of the issuing HIP
stream, so whether a collective sees its input before or after the producing kernel -- and whether the next kernel
sees its output -- depends on timing.  That made the race check (``tests/test_gpu_rehearsal.py``) disagree on cold
runs even with every side stream folded onto the compute stream (``profiles/race_bisect_r4.log``: the first run on a
fresh box differs, the warm reruns agree, independent of which side stream is folded).

``install()`` wraps the ``torch.distributed`` collectives this framework calls so that GPU tensors travel through
host copies: the device-to-host copy of every input is ordered after the current stream's work (and synchronous),
gloo runs on host tensors, and the results are copied back on the current stream -- exactly the stream semantics
RCCL has, so the rehearsal's multi- vs single-stream comparison again tests this framework's own stream / event
ordering.  Sums over 3+ ranks are done in rank order (``_ordered_sum``): gloo's own order follows message arrival.  ``async_op=True`` calls complete before returning (their work handle's ``wait`` is a no-op).  Only the
rehearsal installs this; with RCCL (``nccl``) or CPU gloo nothing is wrapped.  The same for pipeline p2p is
``communicator._HostStagedWork``.
"""
from __future__ import annotations

import functools
from typing import Any, Callable, Optional

import torch
import torch.distributed as dist

_installed = False
_orig: dict[str, Callable[..., Any]] = {}


class _Done:
    """Work handle of a collective that already completed (stream-ordered)."""

    def wait(self, timeout: Any = None) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


def _cuda(t: Any) -> bool:
    return isinstance(t, torch.Tensor) and t.is_cuda


def _host(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to("cpu").contiguous()  # ordered after the current stream's writes of t, synchronous


def _ordered_sum(h: torch.Tensor, group: Any) -> Optional[torch.Tensor]:
    """SUM over ``group`` of the host tensor ``h`` in rank order (None for groups of <= 2 ranks, where gloo's own sum
    is already order-independent).  gloo reduces larger groups in message-arrival order, so fp32 sums of 3+ ranks
    differ from run to run (``profiles/race_repeat_dp4_r4.log``: DP4 runs disagree with every stream folded and any
    GEMM backend); gathering every rank's tensor and adding in rank order makes the result a pure function of the
    inputs, as RCCL's fixed ring order is."""
    n = dist.get_world_size(group)
    if n <= 2:
        return None
    flat = h.contiguous().reshape(-1)
    parts = torch.empty(n * flat.numel(), dtype=h.dtype)
    _orig["all_gather_into_tensor"](parts, flat, group=group)
    parts = parts.view(n, -1)
    out = parts[0].clone()
    for i in range(1, n):
        out += parts[i]
    return out.view(h.shape)


def _is_sum(op: Any) -> bool:
    return op is None or op == dist.ReduceOp.SUM


def _wrap_all_reduce(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(tensor: torch.Tensor, op: Any = None, group: Any = None, async_op: bool = False) -> Any:
        if not _cuda(tensor):
            return orig(tensor, op if op is not None else dist.ReduceOp.SUM, group, async_op)
        h = _host(tensor)
        red = _ordered_sum(h, group) if _is_sum(op) else None
        if red is None:
            orig(h, op if op is not None else dist.ReduceOp.SUM, group)
            red = h
        tensor.copy_(red)
        return _Done() if async_op else None

    return fn


def _wrap_broadcast(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(tensor: torch.Tensor, *args: Any, async_op: bool = False, **kwargs: Any) -> Any:
        if not _cuda(tensor):
            return orig(tensor, *args, async_op=async_op, **kwargs)
        h = _host(tensor)
        orig(h, *args, **kwargs)
        tensor.copy_(h)
        return _Done() if async_op else None

    return fn


def _wrap_reduce_scatter(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(output: torch.Tensor, input: torch.Tensor, op: Any = None, group: Any = None,
           async_op: bool = False) -> Any:
        if not (_cuda(output) or _cuda(input)):
            return orig(output, input, op if op is not None else dist.ReduceOp.SUM, group, async_op)
        hi = _host(input)
        red = _ordered_sum(hi, group) if _is_sum(op) else None
        if red is None:
            ho = torch.empty(output.shape, dtype=output.dtype)
            orig(ho, hi, op if op is not None else dist.ReduceOp.SUM, group)
        else:
            r, n = dist.get_rank(group), output.numel()
            ho = red.reshape(-1)[r * n:(r + 1) * n].reshape(output.shape)
        output.copy_(ho)
        return _Done() if async_op else None

    return fn


def _wrap_all_gather_into(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(output: torch.Tensor, input: torch.Tensor, *args: Any, async_op: bool = False, **kwargs: Any) -> Any:
        if not (_cuda(output) or _cuda(input)):
            return orig(output, input, *args, async_op=async_op, **kwargs)
        ho = torch.empty(output.shape, dtype=output.dtype)
        orig(ho, _host(input), *args, **kwargs)
        output.copy_(ho)
        return _Done() if async_op else None

    return fn


def _wrap_all_gather(orig: Callable[..., Any]) -> Callable[..., Any]:
    """all_gather(tensor_list, tensor, ...)."""

    @functools.wraps(orig)
    def fn(tensor_list: list[torch.Tensor], tensor: torch.Tensor, *args: Any, async_op: bool = False,
           **kwargs: Any) -> Any:
        if not (_cuda(tensor) or any(_cuda(t) for t in tensor_list)):
            return orig(tensor_list, tensor, *args, async_op=async_op, **kwargs)
        hl = [torch.empty(t.shape, dtype=t.dtype) for t in tensor_list]
        orig(hl, _host(tensor), *args, **kwargs)
        for t, h in zip(tensor_list, hl):
            t.copy_(h)
        return _Done() if async_op else None

    return fn


def install() -> None:
    """Routes GPU tensors of the wrapped collectives through host copies (idempotent)."""
    global _installed
    if _installed:
        return
    _installed = True
    for name in ("all_reduce", "broadcast", "reduce_scatter_tensor", "all_gather_into_tensor", "all_gather"):
        _orig[name] = getattr(dist, name)
    dist.all_reduce = _wrap_all_reduce(dist.all_reduce)
    dist.broadcast = _wrap_broadcast(dist.broadcast)
    dist.reduce_scatter_tensor = _wrap_reduce_scatter(dist.reduce_scatter_tensor)
    dist.all_gather_into_tensor = _wrap_all_gather_into(dist.all_gather_into_tensor)
    dist.all_gather = _wrap_all_gather(dist.all_gather)


def installed() -> bool:
    return _installed
