"""Linear layers whose weight gradient is accumulated by the GEMM itself.

With the framework optimizer every trainable parameter's ``.grad`` is a view into one flat gradient
buffer (``OptimizerParamGroup.attach_grads`` tags such parameters with ``_sa_main_grad``).  For those
weights the backward issues ``grad += dY^T X`` as ONE GEMM with a beta=1 epilogue (``ops.gemm.wgrad``: the
hand-written gfx950 weight-gradient kernel, hipBLASLt ``addmm_`` for shapes it does not tile) instead of
materialising ``dW`` and letting autograd add it into ``.grad``: one GEMM, no extra ``[N, K]``
temporary, no elementwise accumulate pass, and a single bf16 rounding of ``grad + dY^T X``.
The optimizer's bucket-ready callback (``_sa_grad_ready``) is invoked in place of autograd's
post-accumulate-grad hook.

A weight may carry ``_sa_grad_row_mask`` (``[N, 1]``, 0/1): rows whose mask is 0 receive no gradient
(LM-head ``finetunable_token_ids``; reference ``transformer/model/layers/lm_head.py:34-53`` masks with a
tensor hook, which a GEMM-accumulated gradient would bypass).  The mask is folded into the output
gradient's columns before the weight-gradient GEMM, so both gradient paths honour it.

Several weights that read the same input (q/k/v, SwiGLU ``dense_in``/``siglu_weight``) run as ONE
GEMM.  When the weights (and their gradients) sit back to back in the flat buffers the combined
``[sum N, K]`` matrix is a zero-copy strided view; otherwise it is concatenated.

Tensor parallelism (column-parallel weights without sequence parallelism): the input gradient must be
summed over the TP group.  Instead of a separate ``copy_to`` region whose all-reduce runs after the whole
linear backward, the Function takes the TP group and issues the all-reduce of ``dX`` asynchronously right
after the dgrad GEMM, runs the weight-gradient GEMM while RCCL moves ``dX`` over xGMI, and waits only
before returning (Megatron's async TP all-reduce; the reference runs them back to back,
``column_parallel_linear.py:137-139``).

Weight-gradient GEMMs are off the backward's critical path (only the optimizer consumes them), so the
GEMM-fused ones can run on a side HIP stream (``SCALING_AMD_WGRAD_STREAM=1``; off by default: measured 2 %
slower on the 7B step, profiles/bench_7b_r2_wgrad_stream_ab.log — concurrent MFMA grids thrash L2/LDS): the next dgrad /
attention / norm kernels of the backward are enqueued without waiting for them, and the hardware fills the
CUs a wgrad grid leaves idle in its last wave with the other stream's workgroups.  Ordering: the side stream
waits for the main stream before each wgrad; the optimizer's bucket reductions wait for the side stream;
an autograd final callback makes the main stream wait for it at the end of every backward, so ``.grad`` is
stream-ordered for any reader after ``backward()`` exactly as without the side stream.

Input gradient ``dX = dY W``: hipBLASLt runs that NN layout at ~1.3 PF/s on gfx950 but the forward's
``X W^T`` layout at ~1.6 PF/s.  With a transposed copy ``W^T`` the backward is ``dY (W^T)^T`` — the forward
layout — so training keeps a transposed copy of every weight (LDS-tiled transpose kernel, ~12 GB for the 7B
model), built once per weight update and reused by every micro-batch.  The copies are keyed by a global
weights generation that the optimizer step, checkpoint loads and LoRA merges advance
(``invalidate_transposed_weights``); ``SCALING_AMD_DGRAD_WT=0`` turns the cache off.
"""
from __future__ import annotations

import os
from typing import Any, Optional, Sequence

import torch
import torch.distributed as dist

from ....ops.attention import stash_gemm
from ....ops.gemm import linear as gemm_linear
from ....ops.gemm import mm, mm_nt, transpose2d, wgrad
from ...utils.debug_env import side_streams_enabled

_GEN = [0]
_WT_MODE = os.environ.get("SCALING_AMD_DGRAD_WT", "1")
_WT_ENABLED = _WT_MODE != "0"
# "all": also small weights (< 1M elements), so every dgrad runs dY (W^T)^T in the forward GEMM layout (tests)
_WT_MIN_NUMEL = 0 if _WT_MODE == "all" else (1 << 20)


_WGRAD_STREAM_ENABLED = os.environ.get("SCALING_AMD_WGRAD_STREAM", "0") == "1"
_wgrad_streams: dict[int, Any] = {}
_sync_queued = [-1]  # autograd graph task id whose end-of-backward sync is queued


def wgrad_stream(device: torch.device) -> Optional[Any]:
    """The side stream of this device's GEMM-fused weight-gradient GEMMs (None when disabled / not on a GPU)."""
    if not _WGRAD_STREAM_ENABLED or device.type != "cuda" or not side_streams_enabled("wgrad"):
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _wgrad_streams.get(idx)
    if st is None:
        st = torch.cuda.Stream(device=idx)
        _wgrad_streams[idx] = st
    return st


def sync_wgrad_stream(device: torch.device) -> None:
    """Makes the current stream wait for every weight-gradient GEMM issued so far on ``device``."""
    if device.type != "cuda":
        return
    st = _wgrad_streams.get(device.index if device.index is not None else torch.cuda.current_device())
    if st is not None:
        torch.cuda.current_stream(device).wait_stream(st)


def _queue_end_of_backward_sync(device: torch.device) -> None:
    # keyed by the autograd graph task: a backward that raised before its final callbacks ran leaves a stale id,
    # which the next backward (a new task id) simply does not match, so its sync is still queued
    task = torch._C._current_graph_task_id()
    if task >= 0 and _sync_queued[0] == task:
        return
    _sync_queued[0] = task

    def _sync() -> None:
        _sync_queued[0] = -1
        sync_wgrad_stream(device)

    torch.autograd.Variable._execution_engine.queue_callback(_sync)


def invalidate_transposed_weights() -> None:
    """Marks every cached W^T stale (call after any in-place change of linear weights)."""
    _GEN[0] += 1


def _transposed(weights: Sequence[torch.Tensor], w: torch.Tensor) -> Optional[torch.Tensor]:
    """Cached contiguous ``w^T`` ([K, sum N]) for the dgrad GEMM, or None where it does not pay."""
    if not (_WT_ENABLED and w.is_cuda and w.dtype in (torch.bfloat16, torch.float16) and w.dim() == 2):
        return None
    if w.shape[0] % 64 or w.shape[1] % 64 or w.numel() < _WT_MIN_NUMEL:
        return None
    key = weights[0]
    c = getattr(key, "_sa_wt_cache", None)
    if c is not None and c[0] == _GEN[0] and c[1] == len(weights) and c[2].shape == (w.shape[1], w.shape[0]):
        return c[2]
    with torch.no_grad():
        wt = transpose2d(w.detach())
    key._sa_wt_cache = (_GEN[0], len(weights), wt)  # type: ignore[attr-defined]
    return wt


def _adjacent(ts: Sequence[Optional[torch.Tensor]]) -> Optional[torch.Tensor]:
    """Zero-copy [sum N, K] view over row-major tensors stored back to back, else None."""
    if any(t is None for t in ts):
        return None
    first = ts[0]
    assert first is not None
    if len(ts) == 1:
        return first if first.is_contiguous() else None
    K = first.shape[-1]
    es = first.element_size()
    nxt = first.data_ptr()
    for t in ts:
        assert t is not None
        if not t.is_contiguous() or t.shape[-1] != K or t.dtype != first.dtype or t.data_ptr() != nxt:
            return None
        if t.untyped_storage().data_ptr() != first.untyped_storage().data_ptr():
            return None
        nxt += t.numel() * es
    rows = sum(t.shape[0] for t in ts)  # type: ignore[union-attr]
    return torch.as_strided(first, (rows, K), (K, 1))


def _rehome_adjacent(weights: Sequence[torch.Tensor]) -> Optional[torch.Tensor]:
    """Moves weights that no optimizer flat buffer owns (inference, frozen base weights) into one contiguous
    buffer, once, so the fused GEMM reads a zero-copy ``[sum N, K]`` view instead of concatenating every call
    (``torch.cat`` of the q/k/v or gate/up weights per forward costs more than the GEMV it feeds)."""
    if any(getattr(w, "_sa_main_grad", False) for w in weights):
        return None
    if len({(w.dtype, w.device, w.shape[-1]) for w in weights}) != 1 or any(w.dim() != 2 for w in weights):
        return None
    with torch.no_grad():
        buf = torch.cat([w.detach() for w in weights], dim=0)
        off = 0
        for w in weights:
            n = w.shape[0]
            w.data = buf[off : off + n]
            off += n
    return _adjacent(weights)


def adjacent_weights(weights: Sequence[torch.Tensor]) -> Optional[torch.Tensor]:
    """Zero-copy ``[sum N, K]`` view over weights that share one input (q/k/v, gate/up), re-homing weights no
    optimizer owns into one buffer on first use; None if they cannot be made adjacent."""
    w = _adjacent(weights)
    if w is None and len(weights) > 1:
        w = _rehome_adjacent(weights)
    return w


def _main_grad_target(weights: Sequence[torch.Tensor]) -> Optional[torch.Tensor]:
    if not all(getattr(w, "_sa_main_grad", False) and w.grad is not None for w in weights):
        return None
    return _adjacent([w.grad for w in weights])


def weight_grads(g2: torch.Tensor, x2: torch.Tensor, weights: Sequence[torch.Tensor], splits: Sequence[int]
                 ) -> list[Optional[torch.Tensor]]:
    """Weight gradients ``dW_i (+)= g2[:, cols_i]^T x2`` of weights sharing the input ``x2``, as ONE GEMM.

    Main-grad weights (all of them attached to the optimizer's flat buffers, stored back to back) get their gradient
    accumulated in place by the GEMM (beta = 0 on the first write of a lazily zeroed step), the optimizer's bucket-ready
    callbacks run, and None is returned for each; otherwise the gradients are returned (split per weight).  Row masks
    (``_sa_grad_row_mask``) are folded into the output-gradient columns first."""
    n = len(weights)
    masks = [getattr(wt, "_sa_grad_row_mask", None) for wt in weights]
    if any(m is not None for m in masks):
        col = torch.cat([m.reshape(-1).to(g2.device, g2.dtype) if m is not None else g2.new_ones(s)
                         for m, s in zip(masks, splits)])
        g2 = g2 * col
    target = _main_grad_target(weights)
    if target is None:
        dw = wgrad(g2, x2)
        return list(torch.split(dw, list(splits), dim=0)) if n > 1 else [dw]
    # lazily zeroed gradients (optimizer ``lazy_grad_zeroing``): the first write of the step overwrites (beta = 0)
    # instead of accumulating into a zeroed buffer
    fresh = [getattr(wt, "_sa_fresh", False) for wt in weights]
    accumulate = not all(fresh)
    for wt, f in zip(weights, fresh):
        if f:
            wt._sa_fresh = False
            if accumulate:
                wt.grad.zero_()
    ws = wgrad_stream(g2.device)
    if ws is not None:
        ws.wait_stream(torch.cuda.current_stream(g2.device))
        with torch.cuda.stream(ws):
            wgrad(g2, x2, target, accumulate=accumulate)
        g2.record_stream(ws)  # keep the operands' memory until the side stream is done
        x2.record_stream(ws)
        _queue_end_of_backward_sync(g2.device)
    else:
        wgrad(g2, x2, target, accumulate=accumulate)
    for wt in weights:
        cb = getattr(wt, "_sa_grad_ready", None)
        if cb is not None:
            cb(wt)
    return [None] * n


class _MultiLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, n: int, want_wt: bool, tp_group: Any,  # type: ignore[override]
                *params: Optional[torch.Tensor]) -> torch.Tensor:
        weights = params[:n]
        biases = params[n:]
        w = _adjacent(weights)
        if w is None:
            w = torch.cat(weights, dim=0)  # type: ignore[arg-type]
        has_bias = len(biases) > 0 and biases[0] is not None
        b = None
        if has_bias:
            b = biases[0] if n == 1 else torch.cat(biases, dim=0)  # type: ignore[arg-type]
        out = stash_gemm(lambda: gemm_linear(x, w, b))
        wt = _transposed(weights, w) if want_wt else None
        ctx.has_wt = wt is not None
        ctx.save_for_backward(x, wt if wt is not None else w, *weights)
        ctx.n, ctx.has_bias, ctx.tp_group = n, has_bias, tp_group
        ctx.splits = [t.shape[0] for t in weights]  # type: ignore[union-attr]
        return out

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        x, w, *weights = ctx.saved_tensors
        n = ctx.n
        dx = None
        work = None
        if ctx.needs_input_grad[0]:
            if ctx.has_wt:  # w is the cached W^T [K, N]: dX = g (W^T)^T in the forward GEMM layout
                dx = mm_nt(g.reshape(-1, g.shape[-1]), w).view(*g.shape[:-1], w.shape[0])
            else:
                dx = mm(g, w)
            if ctx.tp_group is not None:  # TP input-gradient all-reduce overlapped with the wgrad GEMM below
                dx = dx.contiguous()
                work = dist.all_reduce(dx, group=ctx.tp_group, async_op=True)
        dws: list[Optional[torch.Tensor]] = [None] * n
        if any(ctx.needs_input_grad[4 : 4 + n]):
            dws = weight_grads(g.reshape(-1, g.shape[-1]), x.reshape(-1, x.shape[-1]), weights, ctx.splits)
        dbs: list[Optional[torch.Tensor]] = []
        if ctx.has_bias:
            gb = g.reshape(-1, g.shape[-1]).sum(0)
            dbs = list(torch.split(gb, ctx.splits, dim=0)) if n > 1 else [gb]
        if work is not None:
            work.wait()
        return (dx, None, None, None, *dws, *dbs)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, tp_group: Any = None
           ) -> torch.Tensor:
    """``F.linear`` with GEMM-fused gradient accumulation for main-grad weights; ``tp_group``: all-reduce the
    input gradient over it (column-parallel weight, identity forward), overlapped with the wgrad GEMM."""
    want_wt = torch.is_grad_enabled() and x.requires_grad
    if bias is None:
        return _MultiLinear.apply(x, 1, want_wt, tp_group, weight)
    return _MultiLinear.apply(x, 1, want_wt, tp_group, weight, bias)


def multi_linear(x: torch.Tensor, weights: Sequence[torch.Tensor], biases: Optional[Sequence[Optional[torch.Tensor]]] = None,
                 tp_group: Any = None) -> torch.Tensor:
    """``x @ [W_1; ...; W_n]^T (+ [b_1; ...; b_n])`` as one GEMM (forward, dgrad and wgrad)."""
    if len(weights) > 1 and _adjacent(weights) is None:
        _rehome_adjacent(weights)
    want_wt = torch.is_grad_enabled() and x.requires_grad
    if biases is None or any(b is None for b in biases):
        return _MultiLinear.apply(x, len(weights), want_wt, tp_group, *weights)
    return _MultiLinear.apply(x, len(weights), want_wt, tp_group, *weights, *biases)
