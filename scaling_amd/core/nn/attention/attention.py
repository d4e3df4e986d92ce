"""Tensor-parallel self-attention (reference ``src/scaling/core/nn/attention/attention.py:268-796``).

Same constructor, parameter names (``query_key_value`` or ``query``/``key``/``value``, ``dense``,
LoRA ``lora_modules``, ``norm_query``/``norm_key``) and forward signature.  Internals are
MI355X-first:

* activations stay token-major: the projection output ``[b, s, heads*hd]`` *is* ``[T, heads, hd]``,
  so q/k/v are strided views (no ``rearrange`` copies); separate q/k/v weights run as ONE GEMM
  (``fused_column_linear``) with one TP all-reduce in backward;
* RoPE is a HIP kernel applied on those views; attention is the HIP flash kernel (varlen
  ``cu_seqlens``, causal, sliding window incl. mixed local/global heads, GQA without ``repeat_kv``);
* the ``torch`` kernel keeps the reference's dense masked-softmax math (needed for
  attention-score manipulation / AtMan).
"""
from __future__ import annotations

import math
import os
from enum import Enum
from typing import Any, Callable, Optional, Union

import torch

from ....ops import attention as attn_ops
from ....ops._ext import ext, use_native
from ...topology import Topology
from ..linear import ColumnParallelLinear, RowParallelLinear
from ..linear.fused import fused_column_linear
from ..linear.tp_overlap import sp_gather_column
from ..linear.utils import all_concat, all_reduce_scatter_to_sequence_parallel, all_shard
from ..linear.main_grad import adjacent_weights, invalidate_transposed_weights
from ..lora import ParallelLoRa
from ..lora_config import LoRaConfig, LoRAModuleType
from ..masked_softmax import MaskedSoftmax, MaskedSoftmaxConfig, MaskedSoftmaxKernel
from ..norm import LayerNorm, LayerNormConfig, NormType, RMSNorm, get_norm
from ..rotary import RotaryConfig, RotaryEmbedding, RotaryEmbeddingComplex
from ...utils.grad_probe import probe


class RelativePositionEmbeddingType(Enum):
    NONE = "none"
    ROTARY = "rotary"
    ROTARY_COMPLEX = "rotary_complex"


def split_tensor_along_last_dim(tensor: torch.Tensor, num_partitions: int) -> tuple[torch.Tensor, ...]:
    return tuple(torch.split(tensor, tensor.shape[-1] // num_partitions, dim=-1))


def repeat_kv(x: torch.Tensor, n_rep: int) -> torch.Tensor:
    if n_rep == 1:
        return x
    return x.repeat_interleave(n_rep, dim=-2)

# graph-decode step kernels (RoPE + K/V cache append in one launch); SCALING_AMD_DECODE_FUSED=0 for A/B
_DECODE_FUSED = os.environ.get("SCALING_AMD_DECODE_FUSED", "1") != "0"
# graph decode: RMSNorm + q/k/v GEMV + interleaved RoPE + K/V append as ONE launch (ext().gemv_norm_rope)
_DECODE_ROPE_GEMV = _DECODE_FUSED and os.environ.get("SCALING_AMD_DECODE_ROPE_GEMV", "0") == "1"


def get_max_seq_length(cumulative_seq_lengths: torch.Tensor) -> int:
    return int((cumulative_seq_lengths[1:] - cumulative_seq_lengths[:-1]).max().item())


def _segment_ids(cu: torch.Tensor, total: int) -> torch.Tensor:
    """Segment index of every token (number of interior boundaries <= position): a sorted search, which is
    deterministic under ``torch.use_deterministic_algorithms`` (a scatter-add such as ``index_add_`` is not on GPU)."""
    pos = torch.arange(total, dtype=torch.long, device=cu.device)
    if cu.numel() <= 2:
        return torch.zeros_like(pos)
    return torch.searchsorted(cu[1:-1].long().contiguous(), pos, right=True)


def cumulative_seq_lengths_to_dense_attention_mask(
    cumulative_seq_lengths: torch.Tensor, seq_length_per_batch_item: int, causal: bool
) -> torch.Tensor:
    """Boolean mask [b, 1, s, s], True = masked (reference ``attention.py:69-93``), vectorised."""
    total = int(cumulative_seq_lengths[-1].item())
    b = total // seq_length_per_batch_item
    seg = _segment_ids(cumulative_seq_lengths, total).view(b, seq_length_per_batch_item)
    allowed = seg[:, :, None] == seg[:, None, :]
    if causal:
        allowed = torch.tril(allowed)
    return ~allowed.unsqueeze(1)


def multi_head_attention(
    query: torch.Tensor,
    key: torch.Tensor,
    value: torch.Tensor,
    cumulative_seq_lengths: torch.Tensor,
    causal: bool,
    query_key_scaling_factor: float,
    softmax_fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
    dropout_fn: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
    attention_scores_manipulation: Optional[torch.Tensor] = None,
    attentions_score_manipulation_log_additive: Union[bool, list[bool]] = True,
    use_matmul: bool = False,
    cumulative_seq_lengths_key: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """Dense attention on [b, s, n, hd] tensors (k/v already repeated to n heads). Returns [b, s, n*hd]."""
    b, sq, n, hd = query.shape
    sk = key.shape[1]
    q = query.transpose(1, 2)
    k = key.transpose(1, 2)
    v = value.transpose(1, 2)
    scores = torch.matmul(q, k.transpose(-1, -2)) * query_key_scaling_factor  # [b, n, sq, sk]
    if cumulative_seq_lengths_key is None and sq == sk:
        mask = cumulative_seq_lengths_to_dense_attention_mask(cumulative_seq_lengths, sq, causal)
    else:
        # cached decoding: one query block attending to all keys (bottom-right causal alignment)
        qpos = torch.arange(sq, device=q.device)[:, None] + (sk - sq)
        kpos = torch.arange(sk, device=q.device)[None, :]
        mask = (kpos > qpos) if causal else torch.zeros(sq, sk, dtype=torch.bool, device=q.device)
        mask = mask[None, None].expand(b, 1, sq, sk)
    if attention_scores_manipulation is not None:
        flags = (
            [attentions_score_manipulation_log_additive] * b
            if isinstance(attentions_score_manipulation_log_additive, bool)
            else list(attentions_score_manipulation_log_additive)
        )
        rows = []
        for i in range(b):
            si = scores[i]
            if flags[i]:
                si = si + attention_scores_manipulation[i]
            else:
                shift = si.masked_fill(mask[i], 10000.0).min(-1).values.unsqueeze(-1)
                si = (si - shift) * attention_scores_manipulation[i]
            rows.append(si)
        scores = torch.stack(rows)
    probs = softmax_fn(scores, mask)
    if dropout_fn is not None:
        probs = dropout_fn(probs)
    out = torch.matmul(probs.to(v.dtype), v)  # [b, n, sq, hd]
    return out.transpose(1, 2).reshape(b, sq, n * hd)


class KVCache:
    """Preallocated, token-major decode cache ``[capacity, nkv, hd]`` for keys and values.

    The reference grows its cache with one ``torch.cat`` per generated token
    (``src/scaling/core/nn/attention/attention.py:580-588``), which copies the whole history every
    step (O(n^2) HBM traffic over a generation).  Here the buffers are allocated once with headroom
    and doubled when full, so a decode step writes only its new rows; ``append`` returns views of
    the valid prefix, which the flash kernel reads directly (bottom-right causal alignment).
    """

    def __init__(self, k: torch.Tensor, v: torch.Tensor, length: int) -> None:
        self.k, self.v, self.length = k, v, length

    @classmethod
    def start(cls, k: torch.Tensor, v: torch.Tensor, headroom: int = 256) -> "KVCache":
        n = k.shape[0]
        kb = k.new_empty((n + headroom,) + tuple(k.shape[1:]))
        vb = v.new_empty((n + headroom,) + tuple(v.shape[1:]))
        kb[:n].copy_(k)
        vb[:n].copy_(v)
        return cls(kb, vb, n)

    def append(self, k: torch.Tensor, v: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        n, m = self.length, k.shape[0]
        if n + m > self.k.shape[0]:
            cap = max(2 * self.k.shape[0], n + m)
            kb = self.k.new_empty((cap,) + tuple(self.k.shape[1:]))
            vb = self.v.new_empty((cap,) + tuple(self.v.shape[1:]))
            kb[:n].copy_(self.k[:n])
            vb[:n].copy_(self.v[:n])
            self.k, self.v = kb, vb
        self.k[n : n + m].copy_(k)
        self.v[n : n + m].copy_(v)
        self.length = n + m
        return self.k[: self.length], self.v[: self.length]


class DecodeState:
    """Device-resident position of a graph-captured decode loop, shared by every layer's ``StaticKVCache``:
    ``pos`` [1] int64 is the position (= cache row) of the token being fed, ``cu_k`` [2] int32 = [0, pos + 1] the
    key range the flash-decoding kernel reads.  ``advance`` moves both on the device (inside the graph)."""

    def __init__(self, n_prompt: int, device: torch.device) -> None:
        self.pos = torch.full((1,), n_prompt, dtype=torch.long, device=device)
        self.cu_k = torch.tensor([0, n_prompt + 1], dtype=torch.int32, device=device)
        # set by the fused decode kernels when ``pos`` is outside the cache / rotary table (nothing is written then)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)

    def reset(self, n_prompt: int) -> None:
        self.pos.fill_(n_prompt)
        self.cu_k[1:].fill_(n_prompt + 1)
        self.err.zero_()

    def check(self) -> None:
        """Raises if a decode step ran at a position outside its cache (one host read of the error word)."""
        if int(self.err.item()) != 0:
            raise RuntimeError("graph decode: a step's position exceeded the static KV cache or the rotary table; "
                               "its K/V rows were not written")

    def advance(self) -> None:
        self.pos.add_(1)
        self.cu_k[1:].add_(1)


class StaticKVCache:
    """Fixed-capacity decode cache for HIP-graph capture: the new token's K/V rows are written at the device-side
    position (``index_copy_``) and attention reads the whole buffer with a device-side key range, so one decode
    step has the same shapes, pointers and launches at every position (``KVCache`` grows on the host instead)."""

    def __init__(self, k: torch.Tensor, v: torch.Tensor, state: DecodeState) -> None:
        self.k, self.v, self.state = k, v, state

    @classmethod
    def from_cache(cls, kv: "KVCache", capacity: int, state: DecodeState) -> "StaticKVCache":
        n = kv.length
        assert capacity >= n, (capacity, n)
        kb = kv.k.new_zeros((capacity,) + tuple(kv.k.shape[1:]))
        vb = kv.v.new_zeros((capacity,) + tuple(kv.v.shape[1:]))
        kb[:n].copy_(kv.k[:n])
        vb[:n].copy_(kv.v[:n])
        return cls(kb, vb, state)

    def append(self, k: torch.Tensor, v: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        assert k.shape[0] == 1, "graph-captured decoding feeds one token per step"
        self.k.index_copy_(0, self.state.pos, k)
        self.v.index_copy_(0, self.state.pos, v)
        return self.k, self.v, self.state.cu_k


class _LoraUpInto(torch.autograd.Function):
    """``base[:, lo:hi] += scaling * h @ B^T`` for each adapter, as GEMMs accumulating straight into the column
    slices of the q/k/v GEMM output (beta = 1 epilogue: no up-projection tensor, no add pass).  Backward hands
    the slices of the incoming gradient through without the clone autograd makes for in-place ops on views:
    dh = scaling * g[:, lo:hi] @ B, dB = scaling * g[:, lo:hi]^T @ h."""

    @staticmethod
    def forward(ctx: Any, base: torch.Tensor, spec: tuple, *hb: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        n = len(spec)
        hs, bs = hb[:n], hb[n:]
        b2 = base.view(hs[0].shape[0], -1)
        for ((lo, hi), sc), h, w in zip(spec, hs, bs):
            b2[:, lo:hi].addmm_(h, w.t(), alpha=sc)
        ctx.mark_dirty(base)
        ctx.spec = spec
        ctx.save_for_backward(*hs, *bs)
        return base

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        spec = ctx.spec
        n = len(spec)
        saved = ctx.saved_tensors
        hs, bs = saved[:n], saved[n:]
        g2 = g.reshape(hs[0].shape[0], -1)
        dhs, dbs = [], []
        for i, (((lo, hi), sc), h, w) in enumerate(zip(spec, hs, bs)):
            gs = g2[:, lo:hi]
            dhs.append(torch.mm(gs, w) * sc if ctx.needs_input_grad[2 + i] else None)
            dbs.append(torch.mm(gs.t(), h) * sc if ctx.needs_input_grad[2 + n + i] else None)
        return (g, None, *dhs, *dbs)


class ParallelSelfAttention(torch.nn.Module):
    def __init__(
        self,
        hidden_size: int,
        num_attention_heads: int,
        masked_softmax_config: MaskedSoftmaxConfig,
        causal: bool = True,
        num_local_attention_heads: int = 0,
        local_attention_window_size: Optional[int] = None,
        scaling_factor: Optional[float] = None,
        dropout_attention_probs: float = 0.0,
        rotary_config: Optional[RotaryConfig] = None,
        relative_position_embedding_type: RelativePositionEmbeddingType = RelativePositionEmbeddingType.ROTARY,
        bias: bool = True,
        device: Optional[torch.device] = None,
        dtype: torch.dtype = torch.float32,
        topology: Optional[Topology] = None,
        init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
        bitfit_bias_name: Optional[str] = None,
        lora_config: Optional[LoRaConfig] = None,
        norm_type: NormType = NormType.LAYERNORM,
        key_query_norm: bool = False,
        layernorm_config: Optional[LayerNormConfig] = None,
        qkv_in_one: bool = True,
        num_kv_heads: Optional[int] = None,
        use_matmul: bool = False,
    ) -> None:
        super().__init__()
        assert not (topology is not None and device is not None), "cannot specify both device and topology"
        from ..linear.utils import get_device

        self._device = get_device(topology=topology, device=device)
        assert hidden_size % num_attention_heads == 0, "hidden size must be divisible by num_attention_heads"
        self.hidden_size = hidden_size
        self.hidden_size_per_attention_head = hidden_size // num_attention_heads
        self.num_attention_heads = num_attention_heads
        self.causal = causal
        self.lora_config = lora_config
        self.use_flash_attention = masked_softmax_config.kernel == MaskedSoftmaxKernel.FLASH_ATTENTION
        self.masked_softmax_config = masked_softmax_config
        self.num_local_attention_heads = num_local_attention_heads
        self.local_attention_window_size = local_attention_window_size
        mp = 1 if topology is None else topology.config.model_parallel_size
        if num_local_attention_heads > 0:
            assert self.use_flash_attention, "local attention is currently only supported with `flash_attention`."
            assert local_attention_window_size is not None, "`local_attention_window_size` needs to be set"
        assert num_attention_heads % mp == 0, "attention heads must be divisible by model parallel size"
        self.num_attention_heads_per_partition = num_attention_heads // mp
        # heads [0, num_local_attention_heads) of the whole layer are windowed; this TP partition holds heads
        # [rank * hp, (rank + 1) * hp), so mixed local/global heads also work under tensor parallelism (the
        # reference raises NotImplementedError there): the kernels take the window per head
        hp = self.num_attention_heads_per_partition
        rank = 0 if topology is None or mp == 1 else topology.model_parallel_rank
        self.num_local_attention_heads_per_partition = (
            min(max(num_local_attention_heads - rank * hp, 0), hp) if num_local_attention_heads > 0 else 0)
        self.dtype = dtype
        self.qkv_in_one = qkv_in_one
        self.num_kv_heads = num_kv_heads
        if num_kv_heads:
            assert not qkv_in_one, "for a differing number of kv heads, qkv cannot be stored in one"
            self.num_kv_heads_per_partition = num_kv_heads // mp
            self.num_repeat_kv = self.num_attention_heads_per_partition // self.num_kv_heads_per_partition
        else:
            self.num_kv_heads_per_partition = self.num_attention_heads_per_partition
            self.num_repeat_kv = 1
        if lora_config:
            self.lora_merged_state = False
            self.lora_modules = torch.nn.ModuleDict()
            for mt in lora_config.parallel_modules:
                rep = 1 if mt in (LoRAModuleType.DENSE, LoRAModuleType.QUERY) else self.num_repeat_kv
                self.lora_modules[f"{mt.value}_{lora_config.name}"] = ParallelLoRa(
                    in_features=hidden_size,
                    out_features=hidden_size // rep,
                    rank=lora_config.rank,
                    topology=topology,
                    dropout=lora_config.dropout,
                    dtype=dtype,
                    lora_module_type=mt,
                    alpha=lora_config.alpha,
                    bias=lora_config.bias,
                    kaiming_a=lora_config.kaiming_a,
                )
        kw = dict(bias=bias, device=device, dtype=dtype, topology=topology, init_method=init_method,
                  bitfit_bias_name=bitfit_bias_name, parallel_output=True)
        if qkv_in_one:
            self.query_key_value = ColumnParallelLinear(hidden_size, 3 * hidden_size, **kw)
        else:
            self.query = ColumnParallelLinear(hidden_size, hidden_size, **kw)
            self.key = ColumnParallelLinear(hidden_size, hidden_size // self.num_repeat_kv, **kw)
            self.value = ColumnParallelLinear(hidden_size, hidden_size // self.num_repeat_kv, **kw)
        self.use_matmul = use_matmul
        self.scaling_factor = (
            scaling_factor if scaling_factor is not None else 1 / math.sqrt(self.hidden_size_per_attention_head)
        )
        self.rotary_embedding: Optional[Union[RotaryEmbedding, RotaryEmbeddingComplex]] = None
        if relative_position_embedding_type == RelativePositionEmbeddingType.ROTARY:
            assert rotary_config is not None
            self.rotary_embedding = RotaryEmbedding(rotary_config, device=self._device, dtype=dtype)
        elif relative_position_embedding_type == RelativePositionEmbeddingType.ROTARY_COMPLEX:
            assert rotary_config is not None
            self.rotary_embedding = RotaryEmbeddingComplex(rotary_config, device=self._device)
        elif relative_position_embedding_type != RelativePositionEmbeddingType.NONE:
            raise NotImplementedError
        self.key_query_norm = key_query_norm
        self.topology = topology
        self.norm_query: Optional[Union[LayerNorm, RMSNorm]] = None
        self.norm_key: Optional[Union[LayerNorm, RMSNorm]] = None
        if key_query_norm:
            self.norm_query = get_norm(norm_type, layernorm_config, self.hidden_size_per_attention_head,
                                       self._device, dtype, bitfit_bias_name)
            self.norm_key = get_norm(norm_type, layernorm_config, self.hidden_size_per_attention_head,
                                     self._device, dtype, bitfit_bias_name)
        self.dropout_attention_probs = dropout_attention_probs
        self.dropout = torch.nn.Dropout(dropout_attention_probs)
        self.dense = RowParallelLinear(
            hidden_size, hidden_size, bias=bias, topology=topology, dtype=dtype, device=device,
            bitfit_bias_name=bitfit_bias_name, init_method=init_method, parallel_input=True,
            parallel_output=(topology.config.sequence_parallel if topology is not None else False),
        )
        self.masked_softmax = MaskedSoftmax(config=masked_softmax_config)
        self.cache: dict[int, Union["KVCache", tuple[None, None]]] = {}

    # ------------------------------------------------------------------ projections
    def _project(self, x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Returns token-major q [T, nq, hd], k/v [T, nkv, hd] (possibly strided views)."""
        return self._project_base(x)[:3]

    def _project_base(self, x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        """q, k, v views plus the single GEMM output they tile."""
        b, s, _ = x.shape
        T = b * s
        hd, nq, nkv = self.hidden_size_per_attention_head, self.num_attention_heads_per_partition, self.num_kv_heads_per_partition
        base = self.query_key_value(x) if self.qkv_in_one else fused_column_linear(
            x, [self.query, self.key, self.value], self.topology)
        q, k, v = self._split_base(base, T)
        return q, k, v, base

    def _split_base(self, base: torch.Tensor, T: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        if self.qkv_in_one:
            hd, nq = self.hidden_size_per_attention_head, self.num_attention_heads_per_partition
            qkv = base.view(T, nq, 3 * hd)  # per-head interleaved [q|k|v]
            return qkv[..., :hd], qkv[..., hd : 2 * hd], qkv[..., 2 * hd :]
        return self._views(base, T)

    def sp_shard_eligible(self) -> bool:
        """Whether ``project_sp_shard`` applies: sequence parallelism over more than one rank and no unmerged LoRA
        adapters (they read the gathered input)."""
        if self.topology is None or not self.topology.config.sequence_parallel:
            return False
        if self.topology.config.model_parallel_size < 2 or (self.lora_config is not None and not self.lora_merged_state):
            return False
        return True

    def project_sp_shard(self, x: torch.Tensor) -> torch.Tensor:
        """The q/k/v projection of the sequence-parallel token shard ``x`` ([b, s/tp, h]) with its all-gather folded
        into the GEMM and overlapped (``tp_overlap.sp_gather_column``): ``[b, s, (heads + 2 kv heads) hd / tp]``, to be
        passed to ``forward`` as ``projected_base``."""
        mods = [self.query_key_value] if self.qkv_in_one else [self.query, self.key, self.value]
        biases = [getattr(m, "bias_param", None) for m in mods]
        return sp_gather_column(x, [m.weight for m in mods], biases, self.topology)

    def decode_norm_project(self, x: torch.Tensor, norm: torch.nn.Module, position_ids: Optional[torch.Tensor] = None,
                            use_cache: bool = False, reset_cache: bool = False, cache_index: int = 0) -> Optional[dict]:
        """The q/k/v projection of ``norm(x)`` for decode-sized inputs (<= 4 tokens, no autograd graph, bias-free,
        no pending LoRA) as ONE GEMV launch that folds the RMSNorm into its pass over the weights
        (``ext().gemv_norm``; the normalised row stays fp32).  Returns the keyword arguments to pass to ``forward``:
        ``projected_base`` (the projection), or -- graph-captured decoding of one token with interleaved RoPE --
        ``projected_step`` (q rotated, k rotated and v already appended to the static cache by the same launch,
        ``ext().gemv_norm_rope``).  None when the fused path does not apply (the caller runs the norm and the plain
        forward)."""
        if not use_cache or reset_cache:  # real decode steps only (see TransformerLayer.forward)
            return None
        prologue = getattr(norm, "gemv_prologue", None)
        nw = prologue() if prologue is not None and _DECODE_FUSED else None
        if nw is None or x.dim() != 3 or not use_native(x) or not x.is_contiguous():
            return None
        K = x.shape[-1]
        rows = x.numel() // K if K else 0
        if not 0 < rows <= 4:
            return None
        if self.lora_config is not None and not self.lora_merged_state:
            return None
        mods = [self.query_key_value] if self.qkv_in_one else [self.query, self.key, self.value]
        weights = [m.weight for m in mods]
        if torch.is_grad_enabled() and (x.requires_grad or nw[0].requires_grad or any(w.requires_grad for w in weights)):
            return None
        if any(getattr(m, "bias_param", None) is not None for m in mods):
            return None
        w = weights[0] if len(weights) == 1 else adjacent_weights(weights)
        x2 = x.reshape(rows, K)
        if w is None or not ext().gemv_norm_ok(x2, w, nw[0]):
            return None
        step = self._decode_norm_rope_step(x2, nw, w, position_ids, use_cache, reset_cache, cache_index)
        if step is not None:
            return {"projected_step": step}
        _, base = ext().gemv_norm(x2, None, nw[0], nw[1], w, 0)
        return {"projected_base": base.view(*x.shape[:-1], w.shape[0])}

    def _decode_norm_rope_step(self, x2: torch.Tensor, nw: tuple, w: torch.Tensor, position_ids: Optional[torch.Tensor],
                               use_cache: bool, reset_cache: bool, cache_index: int) -> Optional[tuple]:
        """norm + q/k/v GEMV + RoPE + K/V append of one graph-decode token in one launch; None if not applicable."""
        if not (_DECODE_ROPE_GEMV and use_cache and not reset_cache and x2.shape[0] == 1 and not self.key_query_norm
                and not self.qkv_in_one):
            return None
        kv = self.cache.get(cache_index)
        re = self.rotary_embedding
        if not (isinstance(kv, StaticKVCache) and re is not None and re.interleaved and self.use_flash_attention):
            return None
        if position_ids is None or position_ids.numel() != 1 or position_ids.data_ptr() != kv.state.pos.data_ptr():
            return None
        q = ext().gemv_norm_rope(x2, nw[0], nw[1], w, re.cos_table, re.sin_table, kv.state.pos,
                                 self.num_attention_heads_per_partition, self.num_kv_heads_per_partition, re.dimensions,
                                 kv.k, kv.v, kv.state.err)
        if q is None:
            return None
        return q, kv.k, kv.v, kv.state.cu_k

    def _views(self, base: torch.Tensor, T: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        hd, nq, nkv = self.hidden_size_per_attention_head, self.num_attention_heads_per_partition, self.num_kv_heads_per_partition
        out = base.view(T, nq * hd + 2 * nkv * hd)
        q = out[:, : nq * hd].view(T, nq, hd)
        k = out[:, nq * hd : (nq + nkv) * hd].view(T, nkv, hd)
        v = out[:, (nq + nkv) * hd :].view(T, nkv, hd)
        return q, k, v

    def _fused_rope_attention(self, base: torch.Tensor, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                              position_ids: Optional[torch.Tensor], s: int, cumulative_seq_lengths: torch.Tensor,
                              max_seq_length: Optional[int], lora_in_base: bool = False) -> Optional[torch.Tensor]:
        """RoPE + flash attention as one autograd node writing dQKV in place (None if not applicable)."""
        nl = self.num_local_attention_heads
        re = self.rotary_embedding
        if re is None or not self.use_flash_attention or self.key_query_norm:
            return None
        if self.lora_config is not None and not self.lora_merged_state and not lora_in_base:
            return None
        pos = position_ids.reshape(-1) if position_ids is not None else None
        return attn_ops.rope_flash_attention(
            base, q, k, v, re.cos_table, re.sin_table, pos, re.dimensions, s, re.interleaved, cumulative_seq_lengths,
            max_seq_length if max_seq_length is not None else s, self.scaling_factor, self.causal,
            self.local_attention_window_size if nl > 0 else None,
            dropout_p=self.dropout_attention_probs if self.training else 0.0,
            local_heads=self.num_local_attention_heads_per_partition if nl > 0 else None,
            deterministic=self.masked_softmax_config.deterministic_flash_attn_bwd)

    def _lora_gemm_accumulates(self, m: torch.nn.Module) -> bool:
        """An adapter whose up-projection can accumulate into the base output (no biases, no active dropout)."""
        if getattr(m.dense_in, "bias", None) is not None or getattr(m.dense_out, "bias", None) is not None:
            return False
        return not (m.dropout is not None and m.dropout.p > 0 and self.training)

    def _lora_into_base(self, x: torch.Tensor, base: torch.Tensor) -> bool:
        """Unmerged q/k/v adapters at model-parallel size 1 with separate q/k/v weights: ONE down-projection GEMM
        over the concatenated A matrices (x read once; one input-gradient GEMM and one gradient accumulation into
        x instead of three), each scaled up-projection added in place into its column slice of the base q/k/v
        GEMM output — which then takes the fused RoPE + flash path like an adapter-free layer.  Same math as
        ``apply_lora`` (reference ``attention.py`` LoRA branch); False when not applicable."""
        cfg = self.lora_config
        assert cfg is not None
        mp = self.topology.config.model_parallel_size if self.topology is not None else 1
        if self.qkv_in_one or mp > 1 or base._base is not None:  # a view output (biased GEMM) cannot be updated in place
            return False
        mods = [m for n, m in self.lora_modules.items() if n != f"dense_{cfg.name}"]
        if not mods:
            return True
        if not all(self._lora_gemm_accumulates(m) for m in mods):
            return False
        hd, nq, nkv = self.hidden_size_per_attention_head, self.num_attention_heads_per_partition, self.num_kv_heads_per_partition
        cols = {LoRAModuleType.QUERY: (0, nq * hd), LoRAModuleType.KEY: (nq * hd, (nq + nkv) * hd),
                LoRAModuleType.VALUE: ((nq + nkv) * hd, (nq + 2 * nkv) * hd)}
        x2 = x.reshape(-1, x.shape[-1])
        a = torch.cat([m.dense_in.weight for m in mods], dim=0) if len(mods) > 1 else mods[0].dense_in.weight
        h = torch.nn.functional.linear(x2, a.to(x2.dtype))
        hs = h.split([m.dense_in.weight.shape[0] for m in mods], dim=1)
        spec = tuple((cols[m.lora_module_type], m.scaling) for m in mods)
        _LoraUpInto.apply(base, spec, *hs, *[m.dense_out.weight.to(x2.dtype) for m in mods])
        return True

    def apply_lora(self, x: torch.Tensor, query: torch.Tensor, key: torch.Tensor, value: torch.Tensor) -> list[torch.Tensor]:
        assert self.lora_config is not None
        T = x.shape[0] * x.shape[1]
        for name, mod in self.lora_modules.items():
            if name == f"dense_{self.lora_config.name}":
                continue
            out = mod(x).reshape(T, -1, self.hidden_size_per_attention_head)
            if mod.lora_module_type == LoRAModuleType.QUERY:
                query = query + out
            elif mod.lora_module_type == LoRAModuleType.KEY:
                key = key + out
            elif mod.lora_module_type == LoRAModuleType.VALUE:
                value = value + out
        return [query, key, value]

    def _decode_rope_append(self, base: torch.Tensor, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                            position_ids: Optional[torch.Tensor], cache_index: int) -> Optional[tuple]:
        """One-token step of graph-captured decoding: rotate q and k and append k/v at the cache's device-side
        position with ONE kernel (``ext().rope_kv_append``) instead of two RoPE launches and two ``index_copy_``.
        Applies when q/k/v are the [q | k | v] column blocks of one projection row and the token's position ids ARE
        the cache position tensor; None otherwise (the caller runs the unfused ops)."""
        kv = self.cache.get(cache_index)
        re = self.rotary_embedding
        if not (isinstance(kv, StaticKVCache) and re is not None and self.use_flash_attention and use_native(base)):
            return None
        if position_ids is None or position_ids.numel() != 1 or position_ids.data_ptr() != kv.state.pos.data_ptr():
            return None
        hd, nq, nkv = self.hidden_size_per_attention_head, q.shape[1], k.shape[1]
        es = base.element_size()
        if not (base.is_contiguous() and base.numel() == (nq + 2 * nkv) * hd and q.data_ptr() == base.data_ptr()
                and k.data_ptr() == base.data_ptr() + nq * hd * es and v.data_ptr() == base.data_ptr() + (nq + nkv) * hd * es
                and q.stride(1) == hd and k.stride(1) == hd and v.stride(1) == hd):
            return None
        qr = ext().rope_kv_append(base.view(1, nq + 2 * nkv, hd), re.cos_table, re.sin_table, kv.state.pos, nq, nkv,
                                  re.dimensions, re.interleaved, kv.k, kv.v, kv.state.err)
        if qr is None:
            return None
        return qr, kv.k, kv.v, kv.state.cu_k

    # ------------------------------------------------------------------ forward
    def forward(
        self,
        x: torch.Tensor,
        cumulative_seq_lengths: torch.Tensor,
        position_ids: Optional[torch.Tensor],
        cumulative_seq_lengths_key: Optional[torch.Tensor] = None,
        use_cache: bool = False,
        reset_cache: bool = False,
        cache_index: int = 0,
        attention_scores_manipulation: Optional[torch.Tensor] = None,
        attentions_score_manipulation_log_additive: Union[bool, list[bool]] = True,
        max_seq_length: Optional[int] = None,
        projected_base: Optional[torch.Tensor] = None,
        projected_step: Optional[tuple] = None,
    ) -> torch.Tensor:
        """``projected_base``: the q/k/v projection of ``x`` already computed; ``projected_step``: (q, k cache,
        v cache, key cu_seqlens) of a graph-decode token whose RoPE and cache append are done
        (both from ``decode_norm_project``)."""
        # a projection computed outside carries the full token shape (x may be a sequence-parallel shard, see
        # project_sp_shard)
        b, s = (projected_base.shape[0], projected_base.shape[1]) if projected_base is not None else x.shape[:2]
        T = b * s
        hd = self.hidden_size_per_attention_head
        fused_append: Optional[tuple] = None
        probe("attention.input", x)
        if projected_step is not None:  # graph decode: norm + q/k/v GEMV + RoPE + K/V append were one launch
            q, k, v, cumulative_seq_lengths_key = projected_step
            fused_append = projected_step
        else:
            if projected_base is not None:
                base = projected_base
                q, k, v = self._split_base(base, T)
            else:
                q, k, v, base = self._project_base(x)
            lora_pending = self.lora_config is not None and not self.lora_merged_state
            lora_in_base = lora_pending and self._lora_into_base(x, base)
            if lora_in_base:  # fresh views of the updated GEMM output
                q, k, v = self._views(base, T)
            probe("attention.qkv", base)
            if not use_cache and not reset_cache and cumulative_seq_lengths_key is None:
                fused = self._fused_rope_attention(base, q, k, v, position_ids, s, cumulative_seq_lengths, max_seq_length,
                                                   lora_in_base=lora_in_base)
                if fused is not None:
                    return self._output(probe("attention.core", fused).reshape(b, s, -1))
            if lora_pending and not lora_in_base:
                q, k, v = self.apply_lora(x, q, k, v)
            if self.key_query_norm:
                assert self.norm_query is not None and self.norm_key is not None
                q = all_shard(self.norm_query(all_concat(q, dim=1, topology=self.topology)), dim=1, topology=self.topology)
                k = all_shard(self.norm_key(all_concat(k, dim=1, topology=self.topology)), dim=1, topology=self.topology)
            if use_cache and not reset_cache and T == 1 and not self.key_query_norm and _DECODE_FUSED:
                fused_append = self._decode_rope_append(base, q, k, v, position_ids, cache_index)
            if fused_append is not None:  # graph decode: RoPE + K/V cache append in one launch
                q, k, v, cumulative_seq_lengths_key = fused_append
            elif self.rotary_embedding is not None:
                pos = position_ids.reshape(-1) if position_ids is not None else None
                q = self.rotary_embedding.apply_tokens(q, pos, s)
                k = self.rotary_embedding.apply_tokens(k, pos, s)

        if use_cache and fused_append is None:
            if not self.causal:
                raise ValueError("KV caching is only supported for causal attention.")
            assert b == 1, f"KV caching is only supported for batch size 1, got {b}"
            kv = None if reset_cache else self.cache[cache_index]
            if isinstance(kv, StaticKVCache):  # graph-captured decoding: device-side write index and key range
                assert self.use_flash_attention, "graph-captured decoding needs the flash attention kernel"
                k, v, cumulative_seq_lengths_key = kv.append(k, v)
            else:
                if reset_cache:
                    self.cache[cache_index] = KVCache.start(k, v)
                else:
                    assert isinstance(kv, KVCache), "use_cache without a preceding reset_cache"
                    k, v = kv.append(k, v)
                cumulative_seq_lengths_key = torch.tensor([0, k.shape[0]], device=x.device, dtype=torch.int32)
        elif reset_cache:
            self.cache[cache_index] = (None, None)

        Tk = k.shape[0]
        if self.use_flash_attention:
            cu_k = cumulative_seq_lengths_key if cumulative_seq_lengths_key is not None else cumulative_seq_lengths
            # segments never cross a batch row, so the row length bounds every segment: no host sync
            max_q = max_seq_length if max_seq_length is not None else s
            max_k = max_q if cumulative_seq_lengths_key is None else Tk
            nl = self.num_local_attention_heads
            common = dict(
                cu_seqlens_q=cumulative_seq_lengths, cu_seqlens_k=cu_k, max_seqlen_q=max_q, max_seqlen_k=max_k,
                softmax_scale=self.scaling_factor, causal=self.causal, dropout_p=self.dropout_attention_probs,
                training=self.training, deterministic=self.masked_softmax_config.deterministic_flash_attn_bwd,
            )
            # mixed local/global heads: ONE launch, the kernel picks the window per q head (heads [0, nl)
            # windowed) — no second launch, no repeat_kv (reference attention.py:619-667 runs two)
            window = self.local_attention_window_size if nl > 0 else None
            hidden = attn_ops.flash_attention(q, k, v, window=window, **common,
                                              local_heads=self.num_local_attention_heads_per_partition if nl > 0 else None)
            hidden = hidden.reshape(b, s, -1)
        else:
            kr = repeat_kv(k, self.num_repeat_kv).reshape(b, Tk // b, -1, hd)
            vr = repeat_kv(v, self.num_repeat_kv).reshape(b, Tk // b, -1, hd)
            hidden = multi_head_attention(
                q.reshape(b, s, -1, hd), kr, vr, cumulative_seq_lengths, self.causal, self.scaling_factor,
                softmax_fn=self.masked_softmax, dropout_fn=self.dropout,
                attention_scores_manipulation=attention_scores_manipulation,
                attentions_score_manipulation_log_additive=attentions_score_manipulation_log_additive,
                use_matmul=self.use_matmul,
                cumulative_seq_lengths_key=None if Tk == T else cumulative_seq_lengths_key,
            )

        return self._output(hidden)

    def _output(self, hidden: torch.Tensor) -> torch.Tensor:
        dense_lora = None
        mod = None
        if self.lora_config and not self.lora_merged_state and LoRAModuleType.DENSE in self.lora_config.parallel_modules:
            mod = self.lora_modules[f"dense_{self.lora_config.name}"]
            mp = self.topology.config.model_parallel_size if self.topology is not None else 1
            if not (mp == 1 and self._lora_gemm_accumulates(mod)):
                dense_lora = mod(all_concat(hidden, dim=-1, topology=self.topology))
                mod = None
        sp = self.topology is not None and self.topology.config.sequence_parallel
        if sp and mod is None and dense_lora is None:  # reduce-scatter fused with (overlapped by) the dense GEMM
            return self.dense.forward_sequence_parallel(hidden)
        out = self.dense(hidden)
        if mod is not None and out._base is None:  # up-projection GEMM accumulates into the dense output
            h = torch.nn.functional.linear(hidden.reshape(-1, hidden.shape[-1]), mod.dense_in.weight.to(hidden.dtype))
            out = _LoraUpInto.apply(out, (((0, out.shape[-1]), mod.scaling),), h, mod.dense_out.weight.to(hidden.dtype))
        elif mod is not None:
            dense_lora = mod(hidden)
        if dense_lora is not None:
            out = out + dense_lora
        if self.topology is not None and self.topology.config.sequence_parallel:
            out = all_reduce_scatter_to_sequence_parallel(out, self.topology)
        return out

    # ------------------------------------------------------------------ LoRA merge
    def _get_delta_one_q_k_v(self) -> torch.Tensor:
        assert self.lora_config is not None
        w = self.query_key_value.weight
        nq = self.num_attention_heads_per_partition
        hd = self.hidden_size_per_attention_head
        delta = torch.zeros(nq, 3, hd, w.shape[1], dtype=w.dtype, device=w.device)
        idx = {f"query_{self.lora_config.name}": 0, f"key_{self.lora_config.name}": 1, f"value_{self.lora_config.name}": 2}
        for name, mod in self.lora_modules.items():
            if name in idx:
                delta[:, idx[name]] += mod.get_delta_weights().view(nq, hd, -1).to(w.dtype)
        return delta.view_as(w)

    @torch.no_grad()
    def merge_lora_weights(self) -> None:
        assert self.lora_config and self.lora_modules, "Merge of LoRa weights called without proper configuration."
        if self.qkv_in_one:
            keys = {f"{m.value}_{self.lora_config.name}" for m in (LoRAModuleType.KEY, LoRAModuleType.VALUE, LoRAModuleType.QUERY)}
            if keys.intersection(self.lora_modules.keys()):
                self.query_key_value.weight.data += self._get_delta_one_q_k_v()
        else:
            for name, mod in self.lora_modules.items():
                target = name.split("_")[0]
                if target != "dense":
                    getattr(self, target).weight.data += mod.get_delta_weights().to(self.dtype)
        if LoRAModuleType.DENSE in self.lora_config.parallel_modules:
            self.dense.weight.data += self.lora_modules[f"dense_{self.lora_config.name}"].get_delta_weights().to(self.dtype)
        del self.lora_modules
        self.lora_merged_state = True
        invalidate_transposed_weights()
