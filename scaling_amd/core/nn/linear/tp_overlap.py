"""Row-parallel output collectives overlapped with the row-parallel GEMM (TP forward).

A row-parallel linear (attention ``dense``, MLP ``dense_out``) produces partial sums that the TP group must
all-reduce (or, with sequence parallelism, reduce-scatter over tokens) before anything can use them; the
reference runs GEMM then collective back to back (``src/scaling/core/nn/linear/utils.py:80-98,128-192``), so at
TP2 with an 8 x 4096-token micro-batch every layer waits twice for a 256 MiB message over one xGMI link.

Here the tokens are cut into ``chunks`` pieces.  The GEMM of piece i runs on the compute stream; its collective
is enqueued on a per-device TP communication stream behind an event of that GEMM, so RCCL moves piece i over
xGMI while the matrix cores multiply piece i+1.  The compute stream waits for the communication stream once,
at the end.

Sequence parallelism keeps the reference's token partition: rank r owns the r-th contiguous slice of the
flattened ``[b*s]`` tokens.  Piece i therefore gathers, for every rank r, the rows
``r*T/tp + i*T/(tp*chunks) + [0, T/(tp*chunks))`` (a ``[tp, rows, K]`` view of the input), so its reduce-scatter
delivers to rank r exactly the i-th sub-slice of r's final shard, written in place.  The backward is the
standard one: all-gather of the output gradient (SP only), then the GEMM-fused linear backward of ``main_grad``.
"""
from __future__ import annotations

from typing import Any, Optional

import torch
import torch.distributed as dist

from ...utils.debug_env import side_streams_enabled
from .main_grad import _MultiLinear, _transposed

_streams: dict[int, Any] = {}


def _tp_comm_stream(device: torch.device) -> Optional[Any]:
    if device.type != "cuda" or not side_streams_enabled("tp_comm"):
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _streams.get(idx)
    if st is None:
        st = torch.cuda.Stream(device=idx)
        _streams[idx] = st
    return st


def chunked_supported(x: torch.Tensor, size: int, chunks: int, reduce_scatter: bool) -> bool:
    if chunks <= 1 or size <= 1 or x.dim() < 2:
        return False
    tokens = x.numel() // x.shape[-1]
    if reduce_scatter and (x.dim() < 3 or x.shape[-2] % size):
        return False
    return tokens % (size * chunks if reduce_scatter else chunks) == 0


class _RowParallelChunked(torch.autograd.Function):
    """Inputs mirror ``_MultiLinear`` (x, n, want_wt, tp_group, weight) so its backward is reused verbatim."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, n: int, want_wt: bool, tp_group: Any,  # type: ignore[override]
                weight: torch.Tensor, reduce_scatter: bool, chunks: int, group: Any, size: int) -> torch.Tensor:
        K = x.shape[-1]
        N = weight.shape[0]
        T = x.numel() // K
        x2 = x.reshape(T, K)
        wt = _transposed([weight], weight) if want_wt else None
        ctx.has_wt = wt is not None
        ctx.save_for_backward(x, wt if wt is not None else weight, weight)
        ctx.n, ctx.has_bias, ctx.tp_group, ctx.splits = 1, False, None, [N]
        ctx.reduce_scatter, ctx.group, ctx.size = reduce_scatter, group, size
        cs = _tp_comm_stream(x.device)
        main = torch.cuda.current_stream(x.device) if cs is not None else None
        wT = weight.t()
        if reduce_scatter:
            R = T // (size * chunks)
            out = torch.empty((T // size, N), dtype=x.dtype, device=x.device)
            x4 = x2.view(size, chunks, R, K)
        else:
            R = T // chunks
            out = torch.empty((T, N), dtype=x.dtype, device=x.device)
        for i in range(chunks):
            if reduce_scatter:
                part = torch.matmul(x4[:, i], wT)  # [size, R, N]: rank r's rows of this piece, rank-major
                dst = out[i * R : (i + 1) * R]
            else:
                part = out[i * R : (i + 1) * R]
                torch.mm(x2[i * R : (i + 1) * R], wT, out=part)
            if cs is not None:
                assert main is not None
                cs.wait_stream(main)
                with torch.cuda.stream(cs):
                    _collective(part, dst if reduce_scatter else None, group)
                part.record_stream(cs)  # the piece's buffer may not be reused before RCCL has read it
            else:
                _collective(part, dst if reduce_scatter else None, group)
        if cs is not None:
            assert main is not None
            main.wait_stream(cs)
        lead = x.shape[:-1]
        if reduce_scatter:
            return out.view(*lead[:-1], lead[-1] // size, N)
        return out.view(*lead, N)

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        if ctx.reduce_scatter:
            from ....parallel.tp import raw_gather_seq

            g = raw_gather_seq(g.contiguous(), ctx.size, ctx.group)
        res = _MultiLinear.backward(ctx, g)
        return (*res, None, None, None, None)


def _collective(part: torch.Tensor, dst: Optional[torch.Tensor], group: Any) -> None:
    if dst is None:
        dist.all_reduce(part, group=group)
    else:
        dist.reduce_scatter_tensor(dst.reshape(-1), part.reshape(-1), group=group)


def row_parallel_chunked(x: torch.Tensor, weight: torch.Tensor, topology: Any, reduce_scatter: bool,
                         chunks: int) -> torch.Tensor:
    """``all_reduce(x @ W^T)`` (or its sequence-parallel reduce-scatter) in ``chunks`` overlapped pieces."""
    size = topology.config.model_parallel_size
    want_wt = torch.is_grad_enabled() and x.requires_grad
    return _RowParallelChunked.apply(x.contiguous(), 1, want_wt, None, weight, reduce_scatter, chunks,
                                     topology.model_parallel_group, size)
