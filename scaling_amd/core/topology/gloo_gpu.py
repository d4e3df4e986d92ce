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
ordering.  ``async_op=True`` calls complete before returning (their work handle's ``wait`` is a no-op).  Only the
rehearsal installs this; with RCCL (``nccl``) or CPU gloo nothing is wrapped.  The same for pipeline p2p is
``communicator._HostStagedWork``.
"""
from __future__ import annotations

import functools
from typing import Any, Callable

import torch
import torch.distributed as dist

_installed = False


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


def _wrap_inplace(orig: Callable[..., Any]) -> Callable[..., Any]:
    """all_reduce(tensor, ...) / broadcast(tensor, src, ...): one tensor read and written."""

    @functools.wraps(orig)
    def fn(tensor: torch.Tensor, *args: Any, async_op: bool = False, **kwargs: Any) -> Any:
        if not _cuda(tensor):
            return orig(tensor, *args, async_op=async_op, **kwargs)
        h = _host(tensor)
        orig(h, *args, **kwargs)
        tensor.copy_(h)
        return _Done() if async_op else None

    return fn


def _wrap_out_in(orig: Callable[..., Any]) -> Callable[..., Any]:
    """reduce_scatter_tensor(output, input, ...) / all_gather_into_tensor(output, input, ...)."""

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
    for name in ("all_reduce", "broadcast"):
        setattr(dist, name, _wrap_inplace(getattr(dist, name)))
    for name in ("reduce_scatter_tensor", "all_gather_into_tensor"):
        setattr(dist, name, _wrap_out_in(getattr(dist, name)))
    dist.all_gather = _wrap_all_gather(dist.all_gather)


def installed() -> bool:
    return _installed
