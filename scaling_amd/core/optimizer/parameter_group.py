"""Optimizer parameter group on flat, bucketed buffers (mixed precision + ZeRO-1).

API parity with reference ``OptimizerParamGroup`` (``optimizer/parameter_group.py:81-667``):
constructed from ``named_parameters_with_meta`` + ``OptimizerParamGroupConfig`` and initialised by the
``Optimizer``.  Internals are MI355X-first:

* every parameter of the group is a view into ONE flat model-dtype buffer, and ``param.grad`` is a
  view into ONE flat gradient buffer (autograd accumulates in place) — no per-parameter copies;
* the flat space is cut into ``B`` buckets of ``S`` elements (``S`` a multiple of ``2*dp``).
  With ZeRO, data-parallel rank ``r`` owns chunk ``r`` of every bucket, so the gradient sync of a
  bucket is exactly one ``reduce_scatter_tensor`` and the parameter refresh one in-place
  ``all_gather_into_tensor`` — launched per bucket on a side HIP stream as soon as the bucket's
  gradients are final (overlap with backward);
* the fp32 master weights and Adam moments of the owned chunks are flat fp32 buffers updated by
  one fused HIP AdamW launch per bucket that also writes the model-dtype parameter chunk.
Checkpoints stay in the reference's layout-independent per-layer format (see ``Optimizer``).
"""
from __future__ import annotations

from typing import Any, Optional

import torch

from ..nn.parameter_meta import CoreParameterMeta
from .learning_rate_scheduler import LearningRateScheduler
from .parameter_group_config import OptimizerParamGroupConfig

NCCL_START_ALIGNMENT_FACTOR = 2


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _merge_ranges(rs: list[tuple[int, int]]) -> list[tuple[int, int]]:
    out: list[tuple[int, int]] = []
    for a, b in sorted(rs):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


class OptimizerParamGroup:
    def __init__(self, named_parameters_with_meta: list[tuple[str, torch.Tensor, CoreParameterMeta]],
                 config: OptimizerParamGroupConfig):
        self.config = config
        self.learning_rate_scheduler = LearningRateScheduler(config.learning_rate_scheduler)
        self.parameter_names: list[str] = [n for n, _, _ in named_parameters_with_meta]
        self.parameter_metas: list[CoreParameterMeta] = [m for _, _, m in named_parameters_with_meta]
        self.parameters_original: list[torch.Tensor] = [p for _, p, _ in named_parameters_with_meta]
        self.dummy_parameters: list[torch.Tensor] = []
        self.zero = False
        self.lr = config.learning_rate_scheduler.learning_rate
        self.adam_step = 0

    # ------------------------------------------------------------------ layout
    def initialize(self, topology: Any, zero: bool, bucket_numel: int = 2**26) -> None:
        self.topology = topology
        self.zero = zero
        device = topology.device
        if not self.parameters_original:
            dummy = torch.nn.Parameter(torch.zeros(1, dtype=torch.float32, device=device))
            meta = CoreParameterMeta.register_on_parameter(dummy, is_model_parallel=False, layer_index=-1,
                                                           parameter_name="dummy_parameter")
            self.dummy_parameters.append(dummy)
            self.parameter_names, self.parameter_metas, self.parameters_original = ["dummy_parameter"], [meta], [dummy]
        dtypes = {p.dtype for p in self.parameters_original}
        assert len(dtypes) == 1, f"all parameters in a group must share one dtype, got {dtypes}"
        self.dtype = dtypes.pop()
        dp = topology.config.data_parallel_size
        self.dp = dp
        self.dp_rank = topology.data_parallel_rank
        self.shards = dp if zero else 1
        align = NCCL_START_ALIGNMENT_FACTOR * dp
        numel = sum(p.numel() for p in self.parameters_original)
        padded = _round_up(max(numel, 1), align)
        S = min(_round_up(bucket_numel, align), padded)
        B = (padded + S - 1) // S
        self.bucket_size, self.num_buckets, self.numel = S, B, numel
        self.chunk = S // self.shards
        total = B * S
        self.flat_param = torch.zeros(total, dtype=self.dtype, device=device)
        self.flat_grad = torch.zeros(total, dtype=self.dtype, device=device)
        self.param_offsets: list[tuple[int, int]] = []
        off = 0
        with torch.no_grad():
            for p in self.parameters_original:
                n = p.numel()
                self.flat_param[off : off + n].copy_(p.data.reshape(-1))
                p.data = self.flat_param[off : off + n].view_as(p)
                self.param_offsets.append((off, n))
                off += n
        self.attach_grads()
        # owned chunks: bucket b -> flat [b*S + r*chunk, +chunk)  <->  owned [b*chunk, +chunk)
        r = self.dp_rank if zero else 0
        self.owned_flat_starts = [b * S + r * self.chunk for b in range(B)]
        self.master = torch.empty(B * self.chunk, dtype=torch.float32, device=device)
        with torch.no_grad():
            for b, s in enumerate(self.owned_flat_starts):
                self.master[b * self.chunk : (b + 1) * self.chunk].copy_(self.flat_param[s : s + self.chunk])
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self.owned_grad: Optional[torch.Tensor] = None
        if dp > 1:
            self.owned_grad = torch.zeros(B * self.chunk, dtype=torch.float32, device=device)
        # owned ranges of TP-duplicated params (excluded from the grad norm on mp ranks != 0)
        self.dup_owned_ranges = [
            rng for i, m in enumerate(self.parameter_metas) if m.is_model_parallel_duplicate
            for rng in self.owned_ranges(i)
        ]
        # lazy gradient zeroing: tied / TP-constant-tied grads are read by cross-rank reductions before any
        # optimizer hook could materialise them, so they are zeroed eagerly; every other parameter's zeroing is
        # deferred to its first gradient write of the step (see ``zero_grad``)
        self._eager_ranges = _merge_ranges([
            (o, o + n) for (o, n), m in zip(self.param_offsets, self.parameter_metas)
            if m.is_tied or m.tied_grad_on_model_parallel
        ])
        self._lazy_params = [
            p for p, m in zip(self.parameters_original, self.parameter_metas)
            if not (m.is_tied or m.tied_grad_on_model_parallel)
        ]
        # param -> buckets, bucket -> number of params overlapping it
        self.param_buckets: list[list[int]] = []
        self.bucket_param_count = [0] * B
        for o, n in self.param_offsets:
            bs = list(range(o // S, (o + max(n, 1) - 1) // S + 1))
            self.param_buckets.append(bs)
            for b in bs:
                self.bucket_param_count[b] += 1

    def attach_grads(self) -> None:
        for (o, n), p in zip(self.param_offsets, self.parameters_original):
            g = self.flat_grad[o : o + n].view_as(p)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g
            p._sa_main_grad = True  # type: ignore[attr-defined]  # linear layers may addmm_ into .grad

    def owned_ranges(self, param_index: int) -> list[tuple[int, int, int]]:
        """(owned_start, param_local_start, length) pieces of parameter `param_index` owned by this rank."""
        o, n = self.param_offsets[param_index]
        out = []
        for b, fs in enumerate(self.owned_flat_starts):
            lo, hi = max(o, fs), min(o + n, fs + self.chunk)
            if lo < hi:
                out.append((b * self.chunk + (lo - fs), lo - o, hi - lo))
        return out

    def bucket_view(self, buf: torch.Tensor, b: int) -> torch.Tensor:
        return buf[b * self.bucket_size : (b + 1) * self.bucket_size]

    def owned_view(self, buf: torch.Tensor, b: int) -> torch.Tensor:
        return buf[b * self.chunk : (b + 1) * self.chunk]

    def param_chunk_view(self, b: int) -> torch.Tensor:
        s = self.owned_flat_starts[b]
        return self.flat_param[s : s + self.chunk]

    def grad_source(self) -> torch.Tensor:
        """fp32 (reduced) owned gradients, or the model-dtype flat grads when nothing was communicated."""
        return self.owned_grad if self.owned_grad is not None else self.flat_grad

    # ------------------------------------------------------------------ misc API parity
    def set_dummy_grad(self) -> None:
        for p in self.dummy_parameters:
            if p.grad is None:
                p.grad = torch.zeros_like(p)

    def get_learning_rate(self) -> float:
        return self.lr

    def refresh_optimized_params(self, topology: Any = None) -> None:
        with torch.no_grad():
            for b, s in enumerate(self.owned_flat_starts):
                self.owned_view(self.master, b).copy_(self.flat_param[s : s + self.chunk])

    def zero_grad(self, set_to_none: bool = True, lazy: bool = False) -> None:
        """Zeroes the flat gradient buffer.

        ``lazy``: only the eagerly zeroed ranges are cleared now; every other parameter is marked ``_sa_fresh``
        and its stale gradient is never read: the GEMM-fused weight-gradient path writes it with beta = 0
        (``core/nn/linear/main_grad.py``), the optimizer's tensor hook zeroes it right before autograd
        accumulates into it, and ``materialize_fresh`` zeroes whatever received no gradient at all before the
        step reads the buffer.  Saves one full write of the gradient buffer per step and the beta = 1 read
        of zeros in every first weight-gradient GEMM."""
        if not lazy:
            self.flat_grad.zero_()
            for p in self.parameters_original:
                p._sa_fresh = False  # type: ignore[attr-defined]
        else:
            for a, b in self._eager_ranges:
                self.flat_grad[a:b].zero_()
            for p in self._lazy_params:
                p._sa_fresh = True  # type: ignore[attr-defined]
        self.attach_grads()

    def materialize_fresh(self) -> None:
        """Zeroes the gradients of parameters that are still ``_sa_fresh`` (no gradient written this step)."""
        for p in self._lazy_params:
            if getattr(p, "_sa_fresh", False):
                p._sa_fresh = False  # type: ignore[attr-defined]
                p.grad.zero_()  # type: ignore[union-attr]

    def log_state(self) -> None:
        pass
