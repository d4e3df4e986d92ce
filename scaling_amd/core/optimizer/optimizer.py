"""AdamW optimizer with mixed precision, ZeRO-1 and bucketed/overlapped data-parallel gradient sync.

Parity with reference ``Optimizer`` (``optimizer/optimizer.py:37-734``): same public API
(``backward``, ``step`` -> ``OptimizerStepOutput``, ``save_checkpoint``/``load_checkpoint``,
``refresh_optimizer_after_model_change``), same checkpoint files (``optimizer_state_layer_{i}.pt``
keyed by ``CoreParameterMeta.key`` with TP-merged fp32 parameter + ``exp_avg``/``exp_avg_sq``;
``optimizer_state_static_mp_{m}_pp_{p}_dp_{d}.pt`` for ``zero_save_static``), same step semantics
(loss-scaler skip, SP norm-grad all-reduce, global grad-norm over TP/PP/DP without duplicates,
clip to ``gradient_clipping``, AdamW, parameter refresh).

MI355X-first differences:
* ZeRO reduces gradients with a reduce-scatter into the owned shard (the reference all-reduces the
  full gradient) and refreshes parameters with in-place all-gathers, bucket by bucket on a side
  stream, overlapped with the last backward pass;
* norm + overflow of all gradients come from one fused HIP reduction and ONE world all-reduce —
  a single host sync per step (the reference syncs once per parameter);
* the update is one fused HIP AdamW launch per bucket (fp32 master + moments, writes the bf16
  parameter copy in the same pass);
* with ZeRO the parameter all-gather of bucket b is issued on the side stream right after bucket b's
  AdamW and completes asynchronously: each pipeline layer's next forward waits only for the buckets
  holding its parameters (``attach_param_sync``/``wait_param_sync``), so the gather of late layers
  overlaps the forward of early ones;
* the update itself (``overlap_optimizer_step``) runs on that side stream too: bucket by bucket, the
  smallest parameter group (norms) first so layer 0 is ready early, then the gradient zeroing; the next
  forward waits per layer, the next backward for the zeroing.  The bandwidth-bound AdamW passes overlap
  the compute-bound forward GEMMs of the next step instead of running between the two.
"""
from __future__ import annotations

import contextlib
import math
from pathlib import Path
from typing import Any, Optional, Union

import torch
import torch.distributed as dist

from ...ops import optim as optim_ops
from ...parallel import custom_allreduce
from ..logging import logger
from ..nn.linear.main_grad import invalidate_transposed_weights, sync_wgrad_stream, wgrad_stream
from ..nn.parameter_meta import CoreParameterMeta
from ..utils.param_merge import merge_parameter, split_parameter
from ..utils.checkpoint_writer import save_file
from ..utils.debug_env import comm_delay_us, side_streams_enabled
from ..utils.safe_load import safe_load
from .base import BaseOptimizer, OptimizerStepOutput
from .loss_scaler import LossScaler
from .optimizer_config import OptimizerConfig
from .parameter_group import OptimizerParamGroup

_SLOTS = ("exp_avg", "exp_avg_sq")


def _is_sp_norm_param(name: str) -> bool:
    """Norm parameters see only their sequence shard under sequence parallelism: their gradients are summed
    over the TP group before the DP reduction (reference ``optimizer.py:253-260`` selects them by name)."""
    return "norm" in name


class Optimizer(BaseOptimizer):
    def __init__(self, config: OptimizerConfig, parameter_groups: list[OptimizerParamGroup], topology: Any) -> None:
        assert config.method == "adamw", f"Unknown optimization method: {config.method}."
        self.config = config
        self.parameter_groups = parameter_groups
        self.topology = topology
        self._assert_no_parameter_duplicates()
        bucket = min(config.grad_bucket_numel, config.allreduce_bucket_size)
        for g in parameter_groups:
            g.initialize(topology=topology, zero=config.zero, bucket_numel=bucket)
        self.step_index = 0
        self.loss_scaler = LossScaler(config=config.loss_scaler, parameter_groups=parameter_groups)
        self.dp = topology.config.data_parallel_size
        self._gpu = topology.device.type == "cuda"
        self._comm_stream = (torch.cuda.Stream(device=topology.device)
                             if (self._gpu and self.dp > 1 and side_streams_enabled("dp_comm")) else None)
        max_bucket = max(g.bucket_size for g in parameter_groups)
        self._scratch = (
            torch.empty(max_bucket, dtype=torch.float32, device=topology.device)
            if (self.dp > 1 and config.zero) else None
        )
        self._launched: list[set[int]] = [set() for _ in parameter_groups]
        self._pending: list[list[int]] = [list(g.bucket_param_count) for g in parameter_groups]
        self._reported: list[set[int]] = [set() for _ in parameter_groups]
        self._armed = False
        self._deferred = self._deferred_buckets()
        self._ag_events: dict[tuple[int, int], Any] = {}
        self._side_stream: Optional[Any] = None  # overlapped optimizer step without a DP comm stream
        self._zero_event: Optional[Any] = None  # gradient zeroing of the last overlapped step
        self._layer_buckets: dict[int, list[tuple[int, int]]] = {}
        self._hooks = []
        self._fresh_hooks = []
        self._lazy_zero = bool(config.lazy_grad_zeroing)
        if self._lazy_zero:
            for g in parameter_groups:
                for p in g.parameters_original:
                    if p.requires_grad:
                        self._fresh_hooks.append(p.register_hook(self._make_fresh_hook(p)))
        if self.dp > 1 and config.overlap_grad_reduce:
            for gi, g in enumerate(parameter_groups):
                for pi, p in enumerate(g.parameters_original):
                    if p.requires_grad and hasattr(p, "register_post_accumulate_grad_hook"):
                        hook = self._make_hook(gi, pi)
                        self._hooks.append(p.register_post_accumulate_grad_hook(hook))
                        p._sa_grad_ready = hook  # type: ignore[attr-defined]  # GEMM-accumulated grads

    # ------------------------------------------------------------------ bookkeeping
    def _assert_no_parameter_duplicates(self) -> None:
        seen: dict[int, str] = {}
        dups = []
        for g in self.parameter_groups:
            for n, p in zip(g.parameter_names, g.parameters_original):
                if id(p) in seen:
                    dups.append(n)
                seen[id(p)] = n
        assert not dups, f"parameters occurring more than once: {dups}"

    def _deferred_buckets(self) -> list[set[int]]:
        """Buckets that must wait for ReduceTiedGrads / TP-constant grads (and, under sequence parallelism, the
        TP all-reduce of the norm weights' partial gradients) before the DP reduction; every other bucket is
        reduced as soon as its gradients are final, overlapped with the rest of the backward."""
        sp = self.topology.config.sequence_parallel and self.topology.config.model_parallel_size > 1
        out = []
        for g in self.parameter_groups:
            s: set[int] = set()
            for n, m, bs in zip(g.parameter_names, g.parameter_metas, g.param_buckets):
                if m.is_tied or m.tied_grad_on_model_parallel or (sp and _is_sp_norm_param(n)):
                    s.update(bs)
            out.append(s)
        return out

    def _make_hook(self, gi: int, pi: int):
        """Gradient-final notification of parameter `pi`, counted once per armed backward.

        A parameter reports either through the GEMM-fused weight-gradient path (``_sa_grad_ready``,
        called right after the GEMM accumulated into ``.grad``) or through autograd's post-accumulate
        hook.  PyTorch also fires that hook when the backward returned no gradient for the weight —
        exactly the GEMM-fused case — so without de-duplication every such weight would count twice and
        its bucket would be reduced before the rest of its gradients were written."""

        def hook(_p: torch.Tensor) -> None:
            if not self._armed or pi in self._reported[gi]:
                return
            self._reported[gi].add(pi)
            for b in self.parameter_groups[gi].param_buckets[pi]:
                self._pending[gi][b] -= 1
                if self._pending[gi][b] == 0 and b not in self._deferred[gi]:
                    self._launch_bucket(gi, b)

        return hook

    @staticmethod
    def _make_fresh_hook(p: torch.Tensor) -> Any:
        """Runs before autograd accumulates a gradient into ``p.grad``: a lazily zeroed gradient is cleared first."""

        def hook(g: torch.Tensor) -> None:
            if getattr(p, "_sa_fresh", False):
                p._sa_fresh = False  # type: ignore[attr-defined]
                p.grad.zero_()  # type: ignore[union-attr]
            return None

        return hook

    def materialize_fresh_grads(self) -> None:
        """Zeroes the lazily zeroed gradients that received nothing this step (before anything reads them)."""
        for g in self.parameter_groups:
            g.materialize_fresh()

    # ------------------------------------------------------------------ gradient sync
    def _launch_bucket(self, gi: int, b: int) -> None:
        if b in self._launched[gi]:
            return
        self._launched[gi].add(b)
        g = self.parameter_groups[gi]
        group = self.topology.data_parallel_group
        inv = 1.0 / self.dp

        def run() -> None:
            self._debug_delay()
            src = g.bucket_view(g.flat_grad, b)
            out = g.owned_view(g.owned_grad, b)
            if self.config.zero:
                if self.config.grad_reduce_dtype == "bfloat16" and src.dtype == torch.bfloat16:
                    tmp = torch.empty(g.chunk, dtype=src.dtype, device=src.device)
                    dist.reduce_scatter_tensor(tmp, src, group=group)
                    optim_ops.cast_scale_(tmp, out, inv)
                else:
                    scratch = self._scratch[: g.bucket_size]
                    optim_ops.cast_scale_(src, scratch, inv)
                    dist.reduce_scatter_tensor(out, scratch, group=group)
            else:
                optim_ops.cast_scale_(src, out, inv)
                dist.all_reduce(out, group=group)

        if self._comm_stream is not None:
            self._comm_stream.wait_stream(torch.cuda.current_stream(self.topology.device))
            ws = wgrad_stream(self.topology.device)  # GEMM-accumulated grads land on the wgrad side stream
            if ws is not None:
                self._comm_stream.wait_stream(ws)
            with torch.cuda.stream(self._comm_stream):
                run()
        else:
            sync_wgrad_stream(self.topology.device)
            run()

    def _debug_delay(self) -> None:
        """Race-check switch (``SCALING_AMD_COMM_DELAY_US``): a busy-wait kernel on the current (communication)
        stream in front of a collective."""
        us = comm_delay_us()
        if us and self._gpu:
            from ...ops._ext import ext

            ext().spin_us(us)

    def prepare_grad_sync(self) -> None:
        """Called by the engine right before the last micro-batch backward of this stage."""
        if self.dp > 1 and self._hooks:
            self._armed = True
            self._pending = [list(g.bucket_param_count) for g in self.parameter_groups]
            self._launched = [set() for _ in self.parameter_groups]
            self._reported = [set() for _ in self.parameter_groups]

    def finish_grad_sync(self) -> None:
        if self.dp == 1:
            return
        self._armed = False
        for gi, g in enumerate(self.parameter_groups):
            for b in range(g.num_buckets):
                self._launch_bucket(gi, b)
        if self._comm_stream is not None:
            torch.cuda.current_stream(self.topology.device).wait_stream(self._comm_stream)
        self._launched = [set() for _ in self.parameter_groups]

    def allreduce_sequence_parallel_gradients(self) -> None:
        if not self.topology.config.sequence_parallel or self.topology.config.model_parallel_size == 1:
            return
        for g in self.parameter_groups:
            for n, p in zip(g.parameter_names, g.parameters_original):
                if _is_sp_norm_param(n) and p.grad is not None:
                    dist.all_reduce(p.grad, group=self.topology.model_parallel_group)

    # ------------------------------------------------------------------ step
    def zero_grad(self, set_to_none: bool = True, lazy: bool = False) -> None:
        for g in self.parameter_groups:
            g.zero_grad(set_to_none, lazy=lazy and self._lazy_zero)

    def backward(self, loss: torch.Tensor) -> None:
        self.wait_grad_zeroing()
        loss = loss.float()
        if self.topology.config.gradient_accumulation_steps > 1:
            loss = loss / self.topology.config.gradient_accumulation_steps
        self.loss_scaler.scale_loss(loss).backward()

    def _grad_stats(self) -> tuple[float, float]:
        """(global grad-norm^2 of unscaled grads, #non-finite) with one world all-reduce."""
        dev = self.topology.device
        acc = torch.zeros(4, dtype=torch.float32, device=dev)
        inv_scale = 1.0 / self.loss_scaler.current_scale
        mp_rank = self.topology.model_parallel_rank
        for g in self.parameter_groups:
            src = g.grad_source()
            optim_ops.sumsq_nonfinite_(src, acc[0:2], inv_scale, accumulate=True)
            if mp_rank != 0:
                for s, _, n in g.dup_owned_ranges:
                    optim_ops.sumsq_nonfinite_(src[s : s + n], acc[2:4], inv_scale, accumulate=True)
        # third slot: error words of the one-shot TP all-reduce (a peer timeout poisons its output with NaN and
        # sets the word); always present so every rank all-reduces the same shape
        errs = custom_allreduce.pending_error_words()
        err = torch.stack(errs).sum().float() if errs else torch.zeros((), dtype=torch.float32, device=dev)
        vals = torch.stack([acc[0] - acc[2], acc[1], err.to(acc.device)]).double()
        if not self.config.zero and self.dp > 1:
            vals[:2] = vals[:2] / self.dp  # every dp rank holds the full (identical) reduced gradient
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(vals)
        v = vals.tolist()
        if v[2] > 0:
            custom_allreduce.reset_error_words()
            custom_allreduce.disable_all()  # the communicators' epoch state is out of step: RCCL from here on
            raise RuntimeError("one-shot tensor-parallel all-reduce timed out waiting for a peer on some rank; "
                               "its outputs were poisoned (NaN) and this step's gradients are invalid")
        return float(v[0]), float(v[1])

    # ------------------------------------------------------------------ overlapped optimizer step
    def _async_step(self) -> bool:
        return bool(self._gpu and self.config.overlap_optimizer_step and side_streams_enabled("opt_step"))

    def _step_stream(self) -> Any:
        if self._comm_stream is not None:  # AdamW then the ZeRO all-gather of the bucket, in order, on one stream
            return self._comm_stream
        if self._side_stream is None:
            self._side_stream = torch.cuda.Stream(device=self.topology.device)
        return self._side_stream

    def wait_grad_zeroing(self) -> None:
        """The gradient buffers are zeroed on the side stream by an overlapped step: wait before writing them."""
        if self._zero_event is not None:
            torch.cuda.current_stream(self.topology.device).wait_event(self._zero_event)
            self._zero_event = None

    # ------------------------------------------------------------------ parameter all-gather overlap
    def _async_param_gather(self) -> bool:
        return bool(self.config.zero and self.dp > 1 and self._comm_stream is not None and self.config.overlap_param_gather)

    def attach_param_sync(self, layers: Any) -> None:
        """Records, per pipeline layer, the (group, bucket) pairs holding its parameters."""
        where: dict[int, list[tuple[int, int]]] = {}
        for gi, g in enumerate(self.parameter_groups):
            for pi, p in enumerate(g.parameters_original):
                where.setdefault(id(p), []).extend((gi, b) for b in g.param_buckets[pi])
        self._layer_buckets = {}
        for layer in layers:
            keys = sorted({k for p in layer.parameters() for k in where.get(id(p), [])})
            self._layer_buckets[id(layer)] = keys

    def wait_param_sync(self, layer: Optional[Any] = None) -> None:
        """Makes the current stream wait for the pending updates / all-gathers of `layer`'s buckets (all if None)."""
        if layer is None:
            self.wait_grad_zeroing()
        if not self._ag_events:
            return
        if layer is None:
            keys = list(self._ag_events.keys())
        else:
            keys = self._layer_buckets.get(id(layer))
            if keys is None:  # unknown module: be safe
                keys = list(self._ag_events.keys())
        stream = torch.cuda.current_stream(self.topology.device)
        for k in keys:
            ev = self._ag_events.pop(k, None)
            if ev is not None:
                stream.wait_event(ev)

    def _gather_bucket(self, g: OptimizerParamGroup, gi: int, b: int) -> None:
        full = g.bucket_view(g.flat_param, b)
        mine = g.param_chunk_view(b)
        if self._async_param_gather():
            assert self._comm_stream is not None
            self._comm_stream.wait_stream(torch.cuda.current_stream(self.topology.device))
            with torch.cuda.stream(self._comm_stream):
                self._debug_delay()
                dist.all_gather_into_tensor(full, mine, group=self.topology.data_parallel_group)
                ev = torch.cuda.Event()
                ev.record(self._comm_stream)
            self._ag_events[(gi, b)] = ev
        else:
            dist.all_gather_into_tensor(full, mine, group=self.topology.data_parallel_group)

    def step(self) -> OptimizerStepOutput:
        self.wait_param_sync()  # parameters never touched by a forward (frozen / unused) still must land
        sync_wgrad_stream(self.topology.device)  # (also done at the end of every backward)
        self.materialize_fresh_grads()
        self.step_index += 1
        for g in self.parameter_groups:
            g.set_dummy_grad()
        self.allreduce_sequence_parallel_gradients()
        self.finish_grad_sync()
        norm_sq, bad = self._grad_stats()
        overflow = bad > 0 or not math.isfinite(norm_sq)
        ls_out = self.loss_scaler.step(overflow)
        if self.config.loss_scaler.enable and overflow:
            logger.warning("loss scaler encountered overflow, skipping step")
            self.zero_grad(lazy=True)
            return OptimizerStepOutput(None, None, None, ls_out.overflow, ls_out.no_overflow_steps,
                                       ls_out.current_loss_scale, None)
        if overflow:
            raise RuntimeError(f"grad norm is {'nan/inf' if bad > 0 else norm_sq}")
        global_grad_norm = math.sqrt(max(norm_sq, 0.0))
        clip = 1.0
        if self.config.gradient_clipping > 0.0 and global_grad_norm >= self.config.gradient_clipping:
            clip = self.config.gradient_clipping / global_grad_norm
        gscale = clip / self.loss_scaler.current_scale
        debug_dict = self._debug_dict() if self.config.debug_log else None
        learning_rates = {}
        for gi, g in enumerate(self.parameter_groups):
            g.lr = g.learning_rate_scheduler.get_lr(step_index=self.step_index)
            g.adam_step += 1
            learning_rates[g.config.name or f"parameter_group_{gi}"] = g.lr
        overlap = self._async_step()
        ctx: Any = contextlib.nullcontext()
        if overlap:
            side = self._step_stream()
            side.wait_stream(torch.cuda.current_stream(self.topology.device))
            ctx = torch.cuda.stream(side)
        # smallest group first (norm weights / biases of every layer), then the large one bucket by bucket in
        # parameter order, so the first layers' parameters are final first
        order = sorted(range(len(self.parameter_groups)),
                       key=lambda i: self.parameter_groups[i].num_buckets * self.parameter_groups[i].bucket_size)
        with ctx:
            for gi in order:
                g = self.parameter_groups[gi]
                src = g.grad_source()
                for b in range(g.num_buckets):
                    if g.owned_grad is not None:
                        gb = g.owned_view(src, b)
                    else:
                        s = g.owned_flat_starts[b]
                        gb = src[s : s + g.chunk]
                    optim_ops.adamw_step_(
                        g.owned_view(g.master, b), gb, g.owned_view(g.exp_avg, b), g.owned_view(g.exp_avg_sq, b),
                        lr=g.lr, beta1=self.config.beta1, beta2=self.config.beta2, eps=self.config.eps,
                        weight_decay=g.config.weight_decay, step=g.adam_step, grad_scale=gscale,
                        param_out=g.param_chunk_view(b),
                    )
                    if self.config.zero and self.dp > 1:
                        self._gather_bucket(g, gi, b)
                    if overlap and (gi, b) not in self._ag_events:
                        ev = torch.cuda.Event()
                        ev.record(torch.cuda.current_stream(self.topology.device))
                        self._ag_events[(gi, b)] = ev
            self.zero_grad(lazy=True)
            if overlap:
                self._zero_event = torch.cuda.Event()
                self._zero_event.record(torch.cuda.current_stream(self.topology.device))
        invalidate_transposed_weights()
        return OptimizerStepOutput(global_grad_norm, None, learning_rates, ls_out.overflow, ls_out.no_overflow_steps,
                                   ls_out.current_loss_scale, debug_dict)

    def _refresh_params(self) -> None:
        if not self.config.zero or self.dp == 1:
            return
        for gi, g in enumerate(self.parameter_groups):
            for b in range(g.num_buckets):
                self._gather_bucket(g, gi, b)
        self.wait_param_sync()

    def _debug_dict(self) -> dict[str, float]:
        d = {}
        for g in self.parameter_groups:
            for p in g.parameters_original:
                m = p.core_parameter_meta
                name = f"{m.parameter_name}-layer-{m.layer_index}"
                d[f"debug/{name}-norm"] = float(p.float().norm().item())
                if p.grad is not None:
                    d[f"debug/{name}-grad-norm"] = float(p.grad.float().norm().item())
        return d

    def clip_gradients(self, global_grad_norm: float) -> bool:
        return self.config.gradient_clipping > 0.0 and global_grad_norm >= self.config.gradient_clipping

    def refresh_optimizer_after_model_change(self) -> None:
        self.wait_param_sync()
        invalidate_transposed_weights()
        for g in self.parameter_groups:
            g.refresh_optimized_params(self.topology)

    def log_state(self) -> None:
        for g in self.parameter_groups:
            logger.debug(f"lr {g.lr}")

    # ------------------------------------------------------------------ state
    def _torch_param_groups(self) -> list[dict[str, Any]]:
        return [
            {"lr": g.lr, "betas": (self.config.beta1, self.config.beta2), "eps": self.config.eps,
             "weight_decay": g.config.weight_decay, "amsgrad": False, "maximize": False, "foreach": None,
             "capturable": False, "differentiable": False, "fused": None, "params": []}
            for g in self.parameter_groups
        ]

    def state_dict(self) -> dict[str, Any]:
        self.wait_param_sync()
        return {
            "step_index": self.step_index,
            "loss_scaler": self.loss_scaler.state_dict(),
            "parameter_groups": [
                {"parameter_names": g.parameter_names, "parameter_metas": [m.state_dict() for m in g.parameter_metas],
                 "adam_step": g.adam_step, "lr": g.lr, "master": g.master, "exp_avg": g.exp_avg,
                 "exp_avg_sq": g.exp_avg_sq}
                for g in self.parameter_groups
            ],
        }

    def _gather_full(self, g: OptimizerParamGroup, buf: torch.Tensor, b: int) -> torch.Tensor:
        """Full fp32 bucket `b` of an owned-layout buffer (all-gather over dp when sharded)."""
        mine = g.owned_view(buf, b)
        if not self.config.zero or self.dp == 1:
            return mine
        full = torch.empty(g.bucket_size, dtype=buf.dtype, device=buf.device)
        dist.all_gather_into_tensor(full, mine.contiguous(), group=self.topology.data_parallel_group)
        return full

    def _full_param_states(self) -> dict[int, list[tuple[torch.Tensor, dict[str, torch.Tensor]]]]:
        """Per group, per parameter: (fp32 param, {exp_avg, exp_avg_sq}) in this rank's TP shard shape."""
        out = {}
        for gi, g in enumerate(self.parameter_groups):
            res = [(torch.empty(p.shape, dtype=torch.float32), {k: torch.empty(p.shape, dtype=torch.float32) for k in _SLOTS})
                   for p in g.parameters_original]
            flat_views = [(r[0].view(-1), {k: v.view(-1) for k, v in r[1].items()}) for r in res]
            for b in range(g.num_buckets):
                fulls = {"p": self._gather_full(g, g.master, b).cpu(), "exp_avg": self._gather_full(g, g.exp_avg, b).cpu(),
                         "exp_avg_sq": self._gather_full(g, g.exp_avg_sq, b).cpu()}
                bs, be = b * g.bucket_size, (b + 1) * g.bucket_size
                for (o, n), (pv, sv) in zip(g.param_offsets, flat_views):
                    lo, hi = max(o, bs), min(o + n, be)
                    if lo >= hi:
                        continue
                    pv[lo - o : hi - o].copy_(fulls["p"][lo - bs : hi - bs])
                    for k in _SLOTS:
                        sv[k][lo - o : hi - o].copy_(fulls[k][lo - bs : hi - bs])
            out[gi] = res
        return out

    def save_checkpoint(self, directory: Union[Path, str]) -> None:
        self.wait_param_sync()
        directory = Path(directory)
        topo = self.topology
        if self.config.zero and self.config.zero_save_static:
            sd = self.state_dict()
            save_file(sd, str(directory / f"optimizer_state_static_mp_{topo.model_parallel_rank}_pp_{topo.pipe_parallel_rank}_dp_{topo.data_parallel_rank}.pt"))
            return
        if topo.data_parallel_rank != 0 and not self.config.zero:
            return
        states = self._full_param_states()
        by_layer: dict[int, dict[str, Any]] = {}
        groups_meta = self._torch_param_groups()
        for gi, g in enumerate(self.parameter_groups):
            for meta, (pfull, slots) in zip(g.parameter_metas, states[gi]):
                dev = topo.device
                merged = merge_parameter(pfull.to(dev), meta, topo)
                merged_slots = {k: merge_parameter(v.to(dev), meta, topo) for k, v in slots.items()}
                m2 = CoreParameterMeta(
                    local_shape=tuple(merged.shape), is_model_parallel=meta.is_model_parallel,
                    model_parallel_dimension=meta.model_parallel_dimension, layer_index=meta.layer_index,
                    parameter_name=meta.parameter_name, layer_class_name=meta.layer_class_name, is_tied=meta.is_tied,
                    tied_layer_indices=set(meta.tied_layer_indices),
                )
                layers = {meta.layer_index} | (set(meta.tied_layer_indices) if meta.is_tied else set())
                entry = {
                    "parameter": merged,
                    "meta": m2.state_dict(),
                    "optimizer_state": {"step": torch.tensor(float(g.adam_step)), **merged_slots},
                }
                for li in layers:
                    d = by_layer.setdefault(li, {"step_index": self.step_index, "loss_scaler": self.loss_scaler.state_dict(),
                                                 "parameters": {}, "optimizer_param_groups": groups_meta})
                    d["parameters"][m2.key_for_layer(meta.layer_index)] = entry
        if topo.model_parallel_rank == 0 and topo.data_parallel_rank == 0:
            for li, d in by_layer.items():
                save_file(d, str(directory / f"optimizer_state_layer_{li}.pt"))
        logger.info("saved optimizer checkpoint")

    def load_checkpoint(self, directory: Union[Path, str]) -> None:
        self.wait_param_sync()
        directory = Path(directory)
        topo = self.topology
        if self.config.zero and self.config.zero_save_static:
            f = directory / f"optimizer_state_static_mp_{topo.model_parallel_rank}_pp_{topo.pipe_parallel_rank}_dp_{topo.data_parallel_rank}.pt"
            sd = safe_load(f, map_location=topo.device)
            self.step_index = sd["step_index"]
            self.loss_scaler.load_state_dict(sd["loss_scaler"])
            for g, s in zip(self.parameter_groups, sd["parameter_groups"]):
                g.adam_step, g.lr = s["adam_step"], s["lr"]
                g.master.copy_(s["master"])
                g.exp_avg.copy_(s["exp_avg"])
                g.exp_avg_sq.copy_(s["exp_avg_sq"])
            return
        layers = set()
        for g in self.parameter_groups:
            for m in g.parameter_metas:
                layers.add(m.layer_index)
                if m.is_tied:
                    layers.update(m.tied_layer_indices)
        params: dict[str, Any] = {}
        first: Optional[dict[str, Any]] = None
        for li in sorted(layers):
            f = directory / f"optimizer_state_layer_{li}.pt"
            if not f.is_file():
                continue
            d = safe_load(f, map_location="cpu")
            first = first or d
            for _, ps in d["parameters"].items():
                meta = CoreParameterMeta.from_state_dict(ps["meta"])
                for k in meta.possible_keys():
                    params[k] = (meta, ps)
        assert first is not None, f"no optimizer state files found in {directory}"
        self.step_index = first["step_index"]
        self.loss_scaler.load_state_dict(first["loss_scaler"])
        for gi, g in enumerate(self.parameter_groups):
            steps = []
            for pi, meta in enumerate(g.parameter_metas):
                if meta.key not in params:
                    if meta.parameter_name == "dummy_parameter":
                        continue
                    raise RuntimeError(f"missing optimizer state for {meta.key}")
                lmeta, ps = params[meta.key]
                full = ps["parameter"]
                slots = dict(ps["optimizer_state"])
                if lmeta.is_model_parallel and topo.config.model_parallel_size > 1:
                    full = split_parameter(full, lmeta, topo)
                    for k in _SLOTS:
                        slots[k] = split_parameter(slots[k], lmeta, topo)
                steps.append(float(slots["step"]))
                fv = full.reshape(-1).to(g.master.device, torch.float32)
                sv = {k: slots[k].reshape(-1).to(g.master.device, torch.float32) for k in _SLOTS}
                for os_, ps_, n in g.owned_ranges(pi):
                    g.master[os_ : os_ + n].copy_(fv[ps_ : ps_ + n])
                    g.exp_avg[os_ : os_ + n].copy_(sv["exp_avg"][ps_ : ps_ + n])
                    g.exp_avg_sq[os_ : os_ + n].copy_(sv["exp_avg_sq"][ps_ : ps_ + n])
            if steps:
                g.adam_step = int(steps[0])
            if gi < len(first["optimizer_param_groups"]):
                g.lr = first["optimizer_param_groups"][gi].get("lr", g.lr)
        invalidate_transposed_weights()
        logger.info("loaded optimizer checkpoint")
