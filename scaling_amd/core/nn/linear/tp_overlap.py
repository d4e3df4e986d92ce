"""Tensor-parallel collectives overlapped with the GEMMs next to them.

``sp_gather_column`` (sequence parallelism, input side): the all-gather of a norm's token shard is folded into the
column-parallel q/k/v or gate/up GEMM that consumes it -- the GEMM of this rank's own rows runs while the other ranks'
rows arrive, and in the backward the reduce-scatter of the input gradient runs under the weight-gradient GEMM
(``_SPGatherColumn``).

``row_parallel_chunked`` (output side): row-parallel output collectives overlapped with the row-parallel GEMM.

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
from ....ops.gemm import mm, mm_nt
from ...utils.debug_env import side_streams_enabled
from .main_grad import _adjacent, _MultiLinear, _rehome_adjacent, _transposed, weight_grads

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
            # [size, R, N]: rank r's rows of this piece, rank-major, as one contiguous-operand GEMM per rank block.
            # (torch.matmul on the strided [size, R, K] view x4[:, i] -- batch stride chunks*R*K -- faulted on
            # MI355X with an illegal memory access inside the vendor GEMM, profiles/matmul_strided_fault_r5.log)
            part = torch.empty((size, R, N), dtype=x2.dtype, device=x2.device)
            for r in range(size):
                torch.mm(x4[r, i], wT, out=part[r])
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
    # the full-token (rank-major) gradient for the weight-gradient GEMM: each piece is copied into place on the
    # communication stream right behind its all-gather, so the copies run beside the input-gradient GEMMs
    gfull = torch.empty((size, chunks, R, N), dtype=g.dtype, device=g.device)
    for i in range(chunks):
        buf = torch.empty((size, R, N), dtype=g.dtype, device=g.device)
        if cs is not None:
            assert main is not None
            cs.wait_stream(main)
            with torch.cuda.stream(cs):
                dist.all_gather_into_tensor(buf.view(-1), gl[i].reshape(-1), group=group)
                ev = torch.cuda.Event()
                ev.record(cs)
                gfull[:, i].copy_(buf)
            events.append(ev)
        else:
            dist.all_gather_into_tensor(buf.view(-1), gl[i].reshape(-1), group=group)
            gfull[:, i].copy_(buf)
        pieces.append(buf)
    dx = torch.empty((size, chunks, R, K), dtype=g.dtype, device=g.device) if ctx.needs_input_grad[0] else None
    wmat = w.t() if ctx.has_wt else w  # [N, K]
    for i in range(chunks):
        if cs is not None:
            assert main is not None
            main.wait_event(events[i])
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


def _mm_into(a: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], out: torch.Tensor) -> None:
    if a.shape[0] == 0:
        return
    if b is None:
        torch.mm(a, w.t(), out=out)
    else:
        torch.addmm(b, a, w.t(), out=out)


class _SPGatherColumn(torch.autograd.Function):
    """``all_gather_seq(x) @ [W_1; ...; W_n]^T (+ b)``: the sequence-parallel gather of a norm output folded into the
    column-parallel GEMM that consumes it, with the collective overlapped both ways.

    Forward: the all-gather of the token shards runs on the TP communication stream while the GEMM of this rank's OWN
    rows (already local) runs on the compute stream; the other ranks' rows follow once they have arrived.  The gathered
    input is written where ``gather_from_sequence_parallel_region`` would put it (rank-major flattened tokens), so
    every output row lands in place: no permutation, no copy, contiguous GEMM operands.  Backward: the input-gradient
    GEMM over all tokens, then its reduce-scatter (the gather's backward) on the communication stream while the
    weight-gradient GEMM runs (Megatron's overlapped sequence-parallel backward; the reference runs norm gather, GEMM,
    and in the backward GEMMs then reduce-scatter back to back: ``core/nn/linear/utils.py:177-192``)."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, n: int, want_wt: bool, group: Any, size: int, rank: int,  # type: ignore[override]
                *params: Optional[torch.Tensor]) -> torch.Tensor:
        weights, biases = params[:n], params[n:]
        w = _adjacent(weights)
        if w is None:
            w = torch.cat(weights, dim=0)  # type: ignore[arg-type]
        has_bias = len(biases) > 0 and biases[0] is not None
        b = (biases[0] if n == 1 else torch.cat(biases, dim=0)) if has_bias else None  # type: ignore[arg-type]
        K = x.shape[-1]
        Ts = x.numel() // K
        xs = x.reshape(Ts, K)
        T, N = Ts * size, w.shape[0]
        full = torch.empty((T, K), dtype=x.dtype, device=x.device)
        out = torch.empty((T, N), dtype=x.dtype, device=x.device)
        cs = _tp_comm_stream(x.device)
        main = torch.cuda.current_stream(x.device) if cs is not None else None
        if cs is not None:
            assert main is not None
            cs.wait_stream(main)
            with torch.cuda.stream(cs):
                dist.all_gather_into_tensor(full, xs, group=group)
        else:
            dist.all_gather_into_tensor(full, xs, group=group)
        _mm_into(xs, w, b, out[rank * Ts : (rank + 1) * Ts])  # own rows: overlaps the gather
        if cs is not None:
            assert main is not None
            main.wait_stream(cs)
        _mm_into(full[: rank * Ts], w, b, out[: rank * Ts])
        _mm_into(full[(rank + 1) * Ts :], w, b, out[(rank + 1) * Ts :])
        wt = _transposed(weights, w) if want_wt else None
        ctx.has_wt = wt is not None
        ctx.save_for_backward(full, wt if wt is not None else w, *weights)
        ctx.n, ctx.has_bias, ctx.group, ctx.size = n, has_bias, group, size
        ctx.splits = [t.shape[0] for t in weights]  # type: ignore[union-attr]
        ctx.x_shape = x.shape
        lead = list(x.shape[:-1])
        lead[1 if len(lead) > 1 else 0] *= size
        return out.view(*lead, N)

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        full, w, *weights = ctx.saved_tensors
        n, size = ctx.n, ctx.size
        T, K = full.shape
        g2 = g.reshape(T, g.shape[-1])
        shard = None
        cs = _tp_comm_stream(g.device)
        main = torch.cuda.current_stream(g.device) if cs is not None else None
        if ctx.needs_input_grad[0]:
            dx = mm_nt(g2, w) if ctx.has_wt else mm(g2, w)  # [T, K]
            shard = torch.empty((T // size, K), dtype=dx.dtype, device=dx.device)
            if cs is not None:
                assert main is not None
                cs.wait_stream(main)
                with torch.cuda.stream(cs):
                    dist.reduce_scatter_tensor(shard, dx, group=ctx.group)
                dx.record_stream(cs)
            else:
                dist.reduce_scatter_tensor(shard, dx, group=ctx.group)
        dws: list[Optional[torch.Tensor]] = [None] * n
        if any(ctx.needs_input_grad[6 : 6 + n]):
            dws = weight_grads(g2, full, weights, ctx.splits)  # overlaps the reduce-scatter
        dbs: list[Optional[torch.Tensor]] = []
        if ctx.has_bias:
            gb = g2.sum(0)
            dbs = list(torch.split(gb, ctx.splits, dim=0)) if n > 1 else [gb]
        if cs is not None and shard is not None:
            assert main is not None
            main.wait_stream(cs)
        return (None if shard is None else shard.view(ctx.x_shape), None, None, None, None, None, *dws, *dbs)


def sp_gather_column(x: torch.Tensor, weights: list, biases: Optional[list], topology: Any) -> torch.Tensor:
    """``gather_from_sequence_parallel_region(x)`` followed by the column-parallel ``x @ [W_1; ...]^T (+ b)`` of
    ``weights`` as ONE overlapped node (``_SPGatherColumn``); ``x`` is this rank's sequence-parallel token shard."""
    size, rank = topology.config.model_parallel_size, topology.model_parallel_rank
    want_wt = torch.is_grad_enabled() and x.requires_grad
    if len(weights) > 1 and _adjacent(weights) is None:
        _rehome_adjacent(weights)
    if biases is None or any(b is None for b in biases):
        return _SPGatherColumn.apply(x.contiguous(), len(weights), want_wt, topology.model_parallel_group, size, rank,
                                     *weights)
    return _SPGatherColumn.apply(x.contiguous(), len(weights), want_wt, topology.model_parallel_group, size, rank,
                                 *weights, *biases)


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
