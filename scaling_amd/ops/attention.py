"""Flash attention (varlen, causal/sliding-window, GQA-native) on gfx950 MFMA (``csrc/kernels/flash_*.hip``).

Replaces the reference's CUDA ``flash_attn_varlen_func`` dependency (``attention.py:204-259``).
Layout is token-major ``[T, heads, head_dim]`` with arbitrary token/head strides, so q/k/v can be
strided views of the fused QKV projection (no ``rearrange`` copies, no ``repeat_kv``).
Backward is deterministic (dK/dV and dQ each owned by one workgroup, no float atomics) for either value of
``deterministic`` (``MaskedSoftmaxConfig.deterministic_flash_attn_bwd``): on MI355X an atomic-dQ backward is
slower (its dQ adds alone are floored at 108.7 ms per 7B step by the ~1.3 TB/s float-atomic rate,
``tools/atomic_dq_floor.hip``, vs 47 ms for the deterministic dQ pass).
bf16 and fp16 operands run natively (fp32 inputs are computed in bf16).  Attention-probability dropout
(reference ``flash_attn_varlen_func(dropout_p=...)``, ``attention.py:245-258``) is fused: the keep mask
is a counter-based hash of (seed, q head, query token, key token) regenerated in the backward kernels,
so no mask is stored; :func:`dropout_keep_mask` is its exact PyTorch twin.
"""
from __future__ import annotations

import contextlib
import math
import threading
from typing import Callable, Any, Iterator, Optional

import torch

from ._ext import ext, use_native


_M32 = 0xFFFFFFFF


def _mul32(x: torch.Tensor, c: int) -> torch.Tensor:
    """(x * c) mod 2^32 for int64 tensors holding uint32 values, without int64 overflow."""
    lo, hi = c & 0xFFFF, c >> 16
    return (x * lo + (((x * hi) & 0xFFFF) << 16)) & _M32


def _mix32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    return x ^ (x >> 16)


def dropout_threshold(p: float) -> int:
    return min(int(p * 4294967296.0), 0xFFFFFFFF)


def dropout_keep_mask(seed: int, heads: torch.Tensor, q_tokens: torch.Tensor, k_tokens: torch.Tensor,
                      p: float) -> torch.Tensor:
    """Bool keep mask [H, Lq, Lk] of the fused flash-attention dropout (same hash as ``flash_attn.h``):
    keep(h, q, k) = mix(mix(mix(seed ^ h*0x9e3779b9) + q) ^ k*0x85ebca6b) >= p * 2^32 (token indices are
    positions in the packed [T] token dimension)."""
    h = heads.long()
    hs = _mix32((seed & _M32) ^ _mul32(h, 0x9E3779B9))  # [H]
    row = _mix32((hs[:, None] + q_tokens.long()[None, :]) & _M32)  # [H, Lq]
    kk = _mul32(k_tokens.long(), 0x85EBCA6B)  # [Lk]
    return _mix32(row[:, :, None] ^ kk[None, None, :]) >= dropout_threshold(p)


def dropout_seed(device: torch.device) -> int:
    """Draws a 32-bit dropout seed from the device generator without a host<->device sync: the seed is a
    function of the generator's (seed, offset), and the offset is advanced, so activation checkpointing
    (which restores the RNG state before recomputing) and the TP-constant RNG tracker reproduce it."""
    if device.type == "cuda":
        gen = torch.cuda.default_generators[device.index if device.index is not None else torch.cuda.current_device()]
        off = gen.get_offset()
        gen.set_offset(off + 4)
        base = gen.initial_seed()
    else:
        return int(torch.randint(0, 2**31 - 1, (1,)).item())
    return int((base * 0x9E3779B97F4A7C15 + off * 0xBF58476D1CE4E5B9) >> 32) & _M32


def attention_reference(q, k, v, cu_q, cu_k, scale, causal, window=-1, dropout_p: float = 0.0, training=False,
                        dropout_seed_value: Optional[int] = None, local_heads: Optional[int] = None):
    """Dense per-segment fp32 attention (numerical oracle and CPU path). q:[T,Hq,D], k/v:[Tk,Hk,D].
    With ``dropout_seed_value`` the dropout mask is the fused kernel's (:func:`dropout_keep_mask`).
    ``local_heads``: only q heads [0, local_heads) use ``window``, the others attend globally."""
    Hq, Hk = q.shape[1], k.shape[1]
    rep = Hq // Hk
    out = torch.empty(q.shape[0], Hq, v.shape[2], dtype=q.dtype, device=q.device)
    cq, ck = cu_q.tolist(), cu_k.tolist()
    for i in range(len(cq) - 1):
        qs, qe, ks, ke = cq[i], cq[i + 1], ck[i], ck[i + 1]
        if qe == qs:
            continue
        qi = q[qs:qe].float().transpose(0, 1)  # [H, Lq, D]
        ki = k[ks:ke].float().repeat_interleave(rep, dim=1).transpose(0, 1)
        vi = v[ks:ke].float().repeat_interleave(rep, dim=1).transpose(0, 1)
        s = torch.matmul(qi, ki.transpose(1, 2)) * scale
        Lq, Lk = qe - qs, ke - ks
        qpos = torch.arange(Lq, device=q.device)[:, None] + (Lk - Lq)
        kpos = torch.arange(Lk, device=q.device)[None, :]
        ok = torch.ones(Lq, Lk, dtype=torch.bool, device=q.device)
        if causal:
            ok &= kpos <= qpos
        okw = ok.clone()
        if window is not None and window >= 0:
            okw &= kpos >= qpos - window
            if not causal:
                okw &= kpos <= qpos + window
        nl = Hq if local_heads is None or local_heads < 0 else min(local_heads, Hq)
        okh = torch.stack([okw if h < nl else ok for h in range(Hq)])  # [H, Lq, Lk]
        s = s.masked_fill(~okh, float("-inf"))
        p = torch.softmax(s, dim=-1)
        p = torch.nan_to_num(p, nan=0.0)
        if dropout_p > 0 and training:
            if dropout_seed_value is not None:
                keep = dropout_keep_mask(dropout_seed_value, torch.arange(Hq, device=q.device),
                                         torch.arange(qs, qe, device=q.device), torch.arange(ks, ke, device=q.device),
                                         dropout_p)
                p = p * keep / (1.0 - dropout_p)
            else:
                p = torch.nn.functional.dropout(p, dropout_p)
        out[qs:qe] = torch.matmul(p, vi).transpose(0, 1).to(q.dtype)
    return out


class AttentionStash:
    """Flash-attention outputs kept across an activation-checkpointed region (``activation_checkpointing_type:
    every_layer_keep_attention``): the region's first forward records every flash call's output and log-sum-exp,
    and the recompute in the backward replays them in call order instead of running the attention forward again
    (everything else of the layer -- GEMMs, norms, RoPE -- is recomputed as usual).  Costs the attention output +
    LSE per layer in memory; saves one flash forward per layer and step."""

    def __init__(self, keep_gemms: bool = False) -> None:
        self.items: list[Optional[tuple[torch.Tensor, torch.Tensor]]] = []
        self.pos = 0
        # every_layer_save_matmuls: linear-layer GEMM outputs of the first forward (tensor, version at record time)
        self.keep_gemms = keep_gemms
        self.gemms: list[Optional[tuple[torch.Tensor, int]]] = []
        self.gpos = 0


_stash_state = threading.local()


@contextlib.contextmanager
def attention_stash(stash: Optional[AttentionStash], mode: str) -> Iterator[None]:
    """Makes flash-attention calls inside the block record into (``mode='record'``) or replay from
    (``mode='replay'``) ``stash``; ``stash=None`` is a no-op."""
    prev = getattr(_stash_state, "cur", None)
    _stash_state.cur = None if stash is None else (stash, mode)
    try:
        yield
    finally:
        _stash_state.cur = prev


def stash_active() -> bool:
    """Whether a GEMM-keeping checkpoint region (``every_layer_save_matmuls``) is recording or replaying."""
    cur = getattr(_stash_state, "cur", None)
    return cur is not None and bool(cur[0].keep_gemms)


def stash_gemm(compute: Callable[[], torch.Tensor]) -> torch.Tensor:
    """A linear layer's GEMM output through the checkpoint stash (``every_layer_save_matmuls``): the region's first
    forward records ``compute()``'s output, the recompute in the backward returns it instead of running the GEMM again
    (falling back to ``compute()`` when the kept tensor was modified in place since, e.g. a LoRA up-projection
    accumulated into it).  Outside such a region this is just ``compute()``."""
    cur = getattr(_stash_state, "cur", None)
    if cur is None or not cur[0].keep_gemms:
        return compute()
    stash, mode = cur
    if mode == "replay":
        if stash.gpos < len(stash.gemms):
            item = stash.gemms[stash.gpos]
            stash.gemms[stash.gpos] = None  # the rebuilt graph's saved tensors hold it from here on
            stash.gpos += 1
            if item is not None and item[0]._version == item[1]:
                return item[0]
        return compute()
    out = compute()
    kept = out.detach()
    stash.gemms.append((kept, kept._version))
    return out


def _fa_fwd_stashed(q, k, v, cu_q, cu_k, max_q, scale, causal, window, p_drop, seed, local_heads, max_k):
    cur = getattr(_stash_state, "cur", None)
    if cur is not None and cur[1] == "replay":
        stash = cur[0]
        if stash.pos < len(stash.items) and stash.items[stash.pos] is not None:
            o, lse = stash.items[stash.pos]  # type: ignore[misc]
            stash.items[stash.pos] = None  # the replaying node's saved tensors hold them from here on
            stash.pos += 1
            return o.detach(), lse
    o, lse = ext().fa_fwd(q, k, v, cu_q, cu_k, max_q, scale, causal, window, p_drop, seed, local_heads, max_k)
    if cur is not None and cur[1] == "record":
        cur[0].items.append((o.detach(), lse))
    return o, lse


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, q, k, v, cu_q, cu_k, max_q, max_k, scale, causal, window, p_drop=0.0, seed=0,  # type: ignore[override]
                local_heads=-1):
        o, lse = _fa_fwd_stashed(q, k, v, cu_q, cu_k, max_q, scale, causal, window, p_drop, seed, local_heads, max_k)
        ctx.save_for_backward(q, k, v, o, lse, cu_q, cu_k)
        ctx.cfg = (max_q, max_k, scale, causal, window, p_drop, seed, local_heads)
        return o

    @staticmethod
    def backward(ctx: Any, do: torch.Tensor):  # type: ignore[override]
        q, k, v, o, lse, cu_q, cu_k = ctx.saved_tensors
        max_q, max_k, scale, causal, window, p_drop, seed, local_heads = ctx.cfg
        dq, dk, dv = ext().fa_bwd(do, q, k, v, o, lse, cu_q, cu_k, max_q, max_k, scale, causal, window, None, None, None,
                                  p_drop, seed, local_heads)
        return dq, dk, dv, None, None, None, None, None, None, None, None, None, None


def _spec(t: torch.Tensor, base: torch.Tensor) -> tuple:
    return (tuple(t.shape), tuple(t.stride()), t.storage_offset() - base.storage_offset())


def _view(base: torch.Tensor, spec: tuple) -> torch.Tensor:
    shape, stride, off = spec
    return base.as_strided(shape, stride, base.storage_offset() + off)


def _probe_record(name: str, *tensors: Any) -> None:
    """Race-check forensics (``core/utils/grad_probe.record``; a no-op unless probing is on)."""
    from ..core.utils import grad_probe  # deferred: scaling_amd.core imports this module

    grad_probe.record(name, *tensors)


class _RopeFlashAttn(torch.autograd.Function):
    """RoPE on q/k + flash attention over views of ONE projection output (``base``).

    Backward allocates ``dbase`` once: the attention backward writes dq/dk/dv straight into its q/k/v
    slices with the inverse rotation applied in its dQ / dK epilogues (no RoPE pass over dq / dk), so no per-slice
    gradient buffers, zero-fills, slice copies or gradient sums are materialised (autograd's view backward would do
    all of those)."""

    @staticmethod
    def forward(ctx: Any, base, specs, cos, sin, pos, rot_dim, seq_len, interleaved, cu_q, cu_k, max_q, max_k, scale,
                causal, window, p_drop=0.0, seed=0, local_heads=-1):  # type: ignore[override]
        qi, ki, vi = (_view(base, sp) for sp in specs)
        q = ext().rope(qi, cos, sin, pos, rot_dim, seq_len, interleaved, False)
        k = ext().rope(ki, cos, sin, pos, rot_dim, seq_len, interleaved, False)
        o, lse = _fa_fwd_stashed(q, k, vi, cu_q, cu_k, max_q, scale, causal, window, p_drop, seed, local_heads, max_k)
        ctx.save_for_backward(base, q, k, o, lse, cu_q, cu_k, cos, sin, pos)
        _probe_record("rope_flash.saved@fwd", base, q, k, o, lse, pos, cos, sin, cu_q)
        ctx.cfg = (specs, rot_dim, seq_len, interleaved, max_q, max_k, scale, causal, window, p_drop, seed, local_heads)
        return o

    @staticmethod
    def bwd_into(saved: tuple, cfg: tuple, do: torch.Tensor, dq: torch.Tensor, dk: torch.Tensor, dv: torch.Tensor) -> None:
        """The attention backward written into the q/k/v slices (dq, dk, dv) of a dQKV buffer, the inverse rotation of
        dq / dk folded into the dQ / dK epilogues.  ``saved`` is the node's ``ctx.saved_tensors``, unpacked ONCE by the
        caller (under non-reentrant activation checkpointing a second unpack raises).  (A separate method so race
        forensics can wrap it from outside the production code: tools/attn_forensics.py.)"""
        base, q, k, o, lse, cu_q, cu_k, cos, sin, pos = saved
        specs, rot_dim, seq_len, interleaved, max_q, max_k, scale, causal, window, p_drop, seed, local_heads = cfg
        v = _view(base, specs[2])
        ext().fa_bwd(do, q, k, v, o, lse, cu_q, cu_k, max_q, max_k, scale, causal, window, dq, dk, dv, p_drop, seed,
                     local_heads, cos, sin, pos, rot_dim, seq_len, interleaved)

    @staticmethod
    def backward(ctx: Any, do: torch.Tensor):  # type: ignore[override]
        saved = ctx.saved_tensors
        base, q, k, o, lse, cu_q, cu_k, cos, sin, pos = saved
        _probe_record("rope_flash.saved@bwd", base, q, k, o, lse, pos, cos, sin, cu_q)
        _probe_record("rope_flash.do", do)
        specs = ctx.cfg[0]
        dbase = torch.empty_like(base)
        dq, dk, dv = (_view(dbase, sp) for sp in specs)
        _RopeFlashAttn.bwd_into(saved, ctx.cfg, do, dq, dk, dv)
        _probe_record("rope_flash.dbase", dbase)
        return (dbase,) + (None,) * 17


def rope_flash_attention(base: torch.Tensor, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cos: torch.Tensor,
                         sin: torch.Tensor, pos: Optional[torch.Tensor], rot_dim: int, seq_len: int, interleaved: bool,
                         cu_seqlens: torch.Tensor, max_seqlen: int, softmax_scale: float, causal: bool = True,
                         window: Optional[int] = None, dropout_p: float = 0.0,
                         local_heads: Optional[int] = None, deterministic: bool = True) -> Optional[torch.Tensor]:
    """Fused RoPE + flash attention for q/k/v that are views tiling ``base`` exactly (the QKV GEMM output).

    Returns None when the fused path does not apply (CPU tensors, layouts that do not tile ``base``); the
    caller then runs rope and :func:`flash_attention` separately."""
    if not (use_native(base) and base.is_contiguous() and base.dtype in (torch.bfloat16, torch.float16)):
        return None
    if q.numel() + k.numel() + v.numel() != base.numel():
        return None
    for t in (q, k, v):
        if t.untyped_storage().data_ptr() != base.untyped_storage().data_ptr():
            return None
    specs = (_spec(q, base), _spec(k, base), _spec(v, base))
    cq = cu_seqlens.to(torch.int32)
    p = None if pos is None else pos.reshape(-1).long().contiguous()
    win = -1 if window is None else int(window)
    seed = dropout_seed(base.device) if dropout_p > 0.0 else 0
    return _RopeFlashAttn.apply(base, specs, cos, sin, p, int(rot_dim), int(seq_len), bool(interleaved), cq, cq,
                                int(max_seqlen), int(max_seqlen), float(softmax_scale), bool(causal), win,
                                float(dropout_p), seed, -1 if local_heads is None else int(local_heads))


def flash_attention(
    q: torch.Tensor,
    k: torch.Tensor,
    v: torch.Tensor,
    cu_seqlens_q: torch.Tensor,
    cu_seqlens_k: Optional[torch.Tensor] = None,
    max_seqlen_q: Optional[int] = None,
    max_seqlen_k: Optional[int] = None,
    softmax_scale: Optional[float] = None,
    causal: bool = True,
    window: Optional[int] = None,
    dropout_p: float = 0.0,
    training: bool = False,
    local_heads: Optional[int] = None,
    deterministic: bool = True,
) -> torch.Tensor:
    """q: [T, Hq, D]; k, v: [Tk, Hk, D] (unit last stride); cu_seqlens int32 [nseg+1].

    ``local_heads``: with a ``window``, only q heads [0, local_heads) are windowed and the rest attend
    globally — mixed local/global heads in ONE launch (the kernels pick the window per head)."""
    if cu_seqlens_k is None:
        cu_seqlens_k = cu_seqlens_q
        max_seqlen_k = max_seqlen_q
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    win = -1 if window is None else int(window)
    if use_native(q):
        p_drop = float(dropout_p) if training else 0.0
        in_dtype = q.dtype
        if in_dtype not in (torch.bfloat16, torch.float16):
            # as flash-attn (the reference's kernel) does: the MFMA kernels are bf16/fp16 only, and silently
            # computing an fp32 model's attention in bf16 would make an fp32 run useless as an fp32 oracle
            raise TypeError(f"flash attention supports bfloat16 / float16 inputs, got {in_dtype}; "
                            "use masked_softmax.kernel 'torch' for float32 models")
        cq = cu_seqlens_q.to(torch.int32)
        ck = cu_seqlens_k.to(torch.int32)
        if max_seqlen_q is None:
            max_seqlen_q = int((cq[1:] - cq[:-1]).max().item())
        if max_seqlen_k is None:
            max_seqlen_k = int((ck[1:] - ck[:-1]).max().item())
        seed = dropout_seed(q.device) if p_drop > 0.0 else 0
        lh = -1 if local_heads is None else int(local_heads)
        out = _FlashAttn.apply(q, k, v, cq, ck, int(max_seqlen_q), int(max_seqlen_k), float(scale), bool(causal), win,
                               p_drop, seed, lh)
        return out if out.dtype == in_dtype else out.to(in_dtype)
    return attention_reference(q, k, v, cu_seqlens_q, cu_seqlens_k, scale, causal, win, dropout_p, training,
                               local_heads=local_heads)
