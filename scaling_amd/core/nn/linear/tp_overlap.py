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
mirror image: with sequence parallelism the output gradient is all-gathered piece by piece on the TP stream while the
input-gradient GEMMs of the previous piece run (``_sp_backward_chunked``); otherwise it is the GEMM-fused linear
backward of ``main_grad``.
Under ``every_layer_save_matmuls`` the whole piecewise GEMM + collective output goes through the checkpoint stash like
any linear-layer GEMM, so the recompute replays it (no GEMM and no collective on any TP rank).
"""
from __future__ import annotations

from typing import Any, Optional

import torch
import torch.distributed as dist

from ....ops.attention import stash_gemm
from ...utils.debug_env import side_streams_enabled
from .main_grad import _MultiLinear, _transposed, weight_grads

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


def _chunked_forward(x2: torch.Tensor, weight: torch.Tensor, reduce_scatter: bool, chunks: int, group: Any,
                     size: int) -> torch.Tensor:
    """The pieces: GEMM of piece i on the compute stream, its collective on the TP comm stream behind it."""
    T, K = x2.shape
    N = weight.shape[0]
    cs = _tp_comm_stream(x2.device)
    main = torch.cuda.current_stream(x2.device) if cs is not None else None
    wT = weight.t()
    if reduce_scatter:
        R = T // (size * chunks)
        out = torch.empty((T // size, N), dtype=x2.dtype, device=x2.device)
        x4 = x2.view(size, chunks, R, K)
    else:
        R = T // chunks
        out = torch.empty((T, N), dtype=x2.dtype, device=x2.device)
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
    return out


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
        ctx.reduce_scatter, ctx.group, ctx.size, ctx.chunks = reduce_scatter, group, size, chunks
        out = stash_gemm(lambda: _chunked_forward(x2, weight, reduce_scatter, chunks, group, size))
        lead = x.shape[:-1]
        if reduce_scatter:
            return out.view(*lead[:-1], lead[-1] // size, N)
        return out.view(*lead, N)

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        if ctx.reduce_scatter:
            return _sp_backward_chunked(ctx, g)
        res = _MultiLinear.backward(ctx, g)
        return (*res, None, None, None, None)


def _sp_backward_chunked(ctx: Any, g: torch.Tensor) -> tuple:
    """Sequence-parallel backward in the forward's token pieces: the all-gather of output-gradient piece i runs on the
    TP comm stream while the input-gradient GEMMs of piece i-1 run on the compute stream; the weight gradient is ONE
    GEMM over the assembled full-token gradient at the end (its bucket is final only then)."""
    x, w, weight = ctx.saved_tensors
    size, chunks, group = ctx.size, ctx.chunks, ctx.group
    N, K = weight.shape[0], x.shape[-1]
    T = x.numel() // K
    R = T // (size * chunks)
    gl = g.contiguous().view(chunks, R, N)  # this rank's shard; piece i = its i-th sub-slice
    cs = _tp_comm_stream(g.device)
    main = torch.cuda.current_stream(g.device) if cs is not None else None
    pieces, events = [], []
    for i in range(chunks):
        buf = torch.empty((size, R, N), dtype=g.dtype, device=g.device)
        if cs is not None:
            assert main is not None
            cs.wait_stream(main)
            with torch.cuda.stream(cs):
                dist.all_gather_into_tensor(buf.view(-1), gl[i].reshape(-1), group=group)
                ev = torch.cuda.Event()
                ev.record(cs)
            events.append(ev)
        else:
            dist.all_gather_into_tensor(buf.view(-1), gl[i].reshape(-1), group=group)
        pieces.append(buf)
    gfull = torch.empty((size, chunks, R, N), dtype=g.dtype, device=g.device)  # full-token (rank-major) order
    dx = torch.empty((size, chunks, R, K), dtype=g.dtype, device=g.device) if ctx.needs_input_grad[0] else None
    wmat = w.t() if ctx.has_wt else w  # [N, K]
    for i in range(chunks):
        if cs is not None:
            assert main is not None
            main.wait_event(events[i])
        gfull[:, i].copy_(pieces[i])
        if dx is not None:
            for r in range(size):
                torch.mm(pieces[i][r], wmat, out=dx[r, i])
    if cs is not None:
        assert main is not None
        main.wait_stream(cs)
    dws = [None]
    if ctx.needs_input_grad[4]:
        dws = weight_grads(gfull.view(T, N), x.reshape(T, K), [weight], [N])
    return (None if dx is None else dx.view(x.shape), None, None, None, dws[0], None, None, None, None)


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
