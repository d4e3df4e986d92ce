"""Tensor-parallel MLPs (reference ``src/scaling/core/nn/mlp.py:21-167``).

``ParallelSwiGLUMLP`` keeps the reference parameters (``dense_in``, ``siglu_weight``, ``dense_out``)
but runs ``dense_in``/``siglu_weight`` as one fused GEMM whose ``[..., 2F]`` output feeds the HIP
SwiGLU kernel directly (and whose backward receives the fused gradient from that kernel).

With the fused node enabled for its shapes (``ops.gemm.nt_fused_mlp_enabled``; model-parallel size 1, no biases, outside a
GEMM-keeping activation-checkpoint region) the whole MLP is ONE autograd node on the NT kernel's fused epilogues
(``_SwiGLUMLPFused``): the gate/up GEMM writes ``z = [g | u]`` and ``h = silu(g) u`` in one pass, and the backward's
down-projection input gradient consumes ``dh`` in registers and writes ``dz`` directly -- no SwiGLU pass over HBM in
either direction.

Otherwise, where ``ops.gemm.nt_swiglu_bwd_enabled`` picks the shape (opt-in; measured slower in the 7B step), only the
backward is fused:
``_SwiGLUDown`` runs the unfused forward (SwiGLU kernel + hipBLASLt down projection) and computes ``dz`` from the down
projection's input-gradient GEMM with the SwiGLU backward in its epilogue (no dh round trip through HBM, no stand-alone
SwiGLU backward pass).
"""
from __future__ import annotations

from typing import Any, Callable, Optional

import torch

from ...ops import swiglu as swiglu_ops
from ...ops._ext import ext, use_native
from ...ops.attention import stash_active
from ...ops.gemm import linear as gemm_linear
from ...ops.gemm import mm_nt, nt_fused_mlp_enabled, nt_swiglu_bwd_enabled, transpose2d
from ..topology import Topology
from .activation_function import ActivationFunction, get_activation_function
from .linear import ColumnParallelLinear, RowParallelLinear
from .linear.fused import fused_column_linear
from .linear.tp_overlap import sp_gather_column
from .linear.main_grad import _transposed, adjacent_weights, weight_grads


def _intermediate(io_features: int, factor: float) -> int:
    assert float(int(io_features * factor)) == io_features * factor, (
        "io_features * intermediate_feature_factor does not result in a natural number for feature dimensions"
    )
    return int(io_features * factor)


class ParallelMLP(torch.nn.Module):
    def __init__(
        self,
        io_features: int,
        intermediate_feature_factor: float,
        bias: bool = True,
        device: Optional[torch.device] = None,
        dtype: torch.dtype = torch.float32,
        topology: Optional[Topology] = None,
        init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
        bitfit_bias_name: Optional[str] = None,
        activation_function: ActivationFunction = ActivationFunction.GELU,
    ) -> None:
        super().__init__()
        f = _intermediate(io_features, intermediate_feature_factor)
        kw = dict(bias=bias, device=device, dtype=dtype, topology=topology, init_method=init_method,
                  bitfit_bias_name=bitfit_bias_name)
        self.dense_in = ColumnParallelLinear(io_features, f, parallel_output=True, **kw)
        self.dense_out = RowParallelLinear(
            f, io_features, parallel_input=True,
            parallel_output=(topology.config.sequence_parallel if topology is not None else False), **kw
        )
        self.activation_function = get_activation_function(activation_function)
        self.topology = topology

    def forward(self, x: torch.Tensor, sp_shard: bool = False) -> torch.Tensor:
        """``sp_shard``: ``x`` is this rank's sequence-parallel token shard; its gather runs folded into (and overlapped
        with) the ``dense_in`` GEMM (``tp_overlap.sp_gather_column``)."""
        if sp_shard:
            h = self.activation_function(sp_gather_column(x, [self.dense_in.weight], [self.dense_in.bias_param],
                                                          self.topology))
        else:
            h = self.activation_function(self.dense_in(x))
        if self.topology is not None and self.topology.config.sequence_parallel:
            return self.dense_out.forward_sequence_parallel(h)
        return self.dense_out(h)


class _SwiGLUMLPFused(torch.autograd.Function):
    """``y = (silu(x Wg^T) * (x Wu^T)) Wd^T`` (TP 1, bias-free) on the NT GEMM kernel's SwiGLU epilogues.

    Forward: one gate/up GEMM writing z and h, one down-projection GEMM.  Saved: x, z, h and the cached transposes
    (the same activations the unfused MLP keeps).  Backward: ``dz`` straight from the down-projection input-gradient
    GEMM (SwiGLU backward in its epilogue), weight gradients through ``weight_grads`` (GEMM-accumulated main grads),
    ``dx = dz Wgu`` on the cached ``Wgu^T``."""

    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, wg: torch.Tensor, wu: torch.Tensor, wd: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        wgu = adjacent_weights([wg, wu])
        assert wgu is not None
        H = x.shape[-1]
        x2 = x.reshape(-1, H)
        T, F = x2.shape[0], wg.shape[0]
        z = torch.empty(T, 2 * F, device=x.device, dtype=x.dtype)
        h = torch.empty(T, F, device=x.device, dtype=x.dtype)
        ext().gemm_nt_swiglu(x2, wgu, z, h)
        y = mm_nt(h, wd)
        wgut = _transposed([wg, wu], wgu)
        wdt = _transposed([wd], wd)
        if wgut is None:  # transpose cache disabled (SCALING_AMD_DGRAD_WT=0): per-call transposes
            wgut = transpose2d(wgu.detach())
        if wdt is None:
            wdt = transpose2d(wd.detach())
        ctx.save_for_backward(x2, z, h, wgut, wdt, wg, wu, wd)
        ctx.lead = x.shape[:-1]
        return y.view(*x.shape[:-1], wd.shape[0])

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor):  # type: ignore[override]
        x2, z, h, wgut, wdt, wg, wu, wd = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dz = torch.empty_like(z)
        ext().gemm_nt_swiglu_bwd(dy2, wdt, z, dz)
        dwd = weight_grads(dy2, h, [wd], [wd.shape[0]])[0] if ctx.needs_input_grad[3] else None
        dx = mm_nt(dz, wgut).view(*ctx.lead, x2.shape[1]) if ctx.needs_input_grad[0] else None
        dwg = dwu = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dwg, dwu = weight_grads(dz, x2, [wg, wu], [wg.shape[0], wu.shape[0]])
        return dx, dwg, dwu, dwd


class _SwiGLUDown(torch.autograd.Function):
    """``y = swiglu(z) Wd^T`` (TP 1, bias-free) whose backward computes ``dz`` straight from the down-projection input
    gradient GEMM (the NT kernel's SwiGLU-backward epilogue: dh never goes to HBM, no stand-alone SwiGLU backward).
    The forward is the unfused one (SwiGLU kernel + hipBLASLt GEMM).  Saved: z and h, the activations the unfused pair
    of nodes keeps."""

    @staticmethod
    def forward(ctx: Any, z: torch.Tensor, wd: torch.Tensor, wdt: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        F = z.shape[-1] // 2
        z2 = z.reshape(-1, 2 * F)
        h = ext().swiglu_fwd(z2[:, :F], z2[:, F:])
        y = gemm_linear(h, wd)
        ctx.save_for_backward(z2, h, wdt, wd)
        ctx.lead = z.shape[:-1]
        return y.view(*z.shape[:-1], wd.shape[0])

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor):  # type: ignore[override]
        z2, h, wdt, wd = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        if not ext().gemm_nt_ok(dy2, wdt):  # e.g. a misaligned view: a fresh copy always qualifies
            dy2 = dy2.clone()
        dz = torch.empty_like(z2)
        ext().gemm_nt_swiglu_bwd(dy2, wdt, z2, dz)
        dwd = weight_grads(dy2, h, [wd], [wd.shape[0]])[0] if ctx.needs_input_grad[1] else None
        return dz.view(*ctx.lead, z2.shape[1]), dwd, None


class ParallelSwiGLUMLP(torch.nn.Module):
    def __init__(
        self,
        io_features: int,
        intermediate_feature_factor: float,
        bias: bool = True,
        device: Optional[torch.device] = None,
        dtype: torch.dtype = torch.float32,
        topology: Optional[Topology] = None,
        init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
        bitfit_bias_name: Optional[str] = None,
    ) -> None:
        super().__init__()
        self.topology = topology
        f = _intermediate(io_features, intermediate_feature_factor)
        kw = dict(bias=bias, device=device, dtype=dtype, topology=topology, init_method=init_method,
                  bitfit_bias_name=bitfit_bias_name)
        self.dense_in = ColumnParallelLinear(io_features, f, parallel_output=True, **kw)
        self.siglu_weight = ColumnParallelLinear(io_features, f, parallel_output=True, **kw)
        self.dense_out = RowParallelLinear(
            f, io_features, parallel_input=True,
            parallel_output=(topology.config.sequence_parallel if topology is not None else False), **kw
        )

    def _decode_weights(self, x: torch.Tensor, residual: torch.Tensor) -> Optional[tuple[torch.Tensor, torch.Tensor]]:
        """``([gate; up], down)`` weights for the decode GEMV path (<= 4 rows, no autograd graph, TP 1, bias-free,
        GEMV-compatible layouts), None when it does not apply."""
        K = x.shape[-1]
        rows = x.numel() // K if K else 0
        if not (0 < rows <= 4 and use_native(x) and residual.shape == x.shape[:-1] + (self.dense_out.out_features,)):
            return None
        if self.topology is not None and self.topology.config.model_parallel_size > 1:
            return None
        params = (self.dense_in.weight, self.siglu_weight.weight, self.dense_out.weight)
        if torch.is_grad_enabled() and (x.requires_grad or residual.requires_grad or any(p.requires_grad for p in params)):
            return None
        if any(getattr(m, "bias_param", None) is not None for m in (self.dense_in, self.siglu_weight, self.dense_out)):
            return None
        w = adjacent_weights([self.dense_in.weight, self.siglu_weight.weight])
        wo = self.dense_out.weight
        if (w is None or not ext().gemv_ok(x.reshape(rows, K), w) or wo.dtype != w.dtype or wo.stride(1) != 1
                or wo.stride(0) % 8 or wo.shape[1] != w.shape[0] // 2 or wo.shape[1] % 8 or wo.data_ptr() % 16):
            return None
        return w, wo

    def decode_forward_residual(self, x: torch.Tensor, residual: torch.Tensor) -> Optional[torch.Tensor]:
        """``residual + self(x)`` for decode-sized inputs (<= 4 tokens, no autograd graph, TP 1, bias-free) as two
        GEMV launches with fused epilogues -- gate/up GEMV + SwiGLU, down GEMV + residual add -- bit-identical to
        the unfused GEMV / SwiGLU / add sequence; None when the fused path does not apply."""
        ws = self._decode_weights(x, residual)
        if ws is None:
            return None
        rows = x.numel() // x.shape[-1]
        h = ext().gemv_swiglu(x.reshape(rows, -1), ws[0])
        return ext().gemv_residual(h, ws[1], residual.reshape(rows, -1)).view(residual.shape)

    def decode_forward_norm(self, h: torch.Tensor, residual: torch.Tensor, norm: torch.nn.Module) -> Optional[torch.Tensor]:
        """``s + self(norm(s))`` with ``s = residual + h`` (the post-attention residual add, RMSNorm and MLP of a
        decode step) as two GEMV launches: the gate/up GEMV folds the add + RMSNorm into its pass over the weights
        (the normalised row stays fp32 instead of being rounded to bf16) and applies SwiGLU, the down GEMV adds
        ``s``.  None when the fused path does not apply."""
        prologue = getattr(norm, "gemv_prologue", None)
        nw = prologue() if prologue is not None else None
        if nw is None or h.shape != residual.shape or not residual.is_contiguous() or not h.is_contiguous():
            return None
        ws = self._decode_weights(h, residual)
        if ws is None:
            return None
        if torch.is_grad_enabled() and nw[0].requires_grad:
            return None
        rows = h.numel() // h.shape[-1]
        h2 = h.reshape(rows, -1)
        if not ext().gemv_norm_ok(h2, ws[0], nw[0]):
            return None
        s, a = ext().gemv_norm(h2, residual.reshape(rows, -1), nw[0], nw[1], ws[0], 2)
        return ext().gemv_residual(a, ws[1], s).view(residual.shape)

    def _fused_eligible(self, x: torch.Tensor) -> bool:
        """The one-node MLP on the NT kernel's SwiGLU epilogues applies: GPU bf16, TP 1, bias-free, adjacent gate/up
        weights, shapes the kernel tiles and the dispatch policy enables, no GEMM-keeping checkpoint region."""
        if not (use_native(x) and x.dtype == torch.bfloat16 and torch.is_grad_enabled()):
            return False
        if self.topology is not None and self.topology.config.model_parallel_size > 1:
            return False
        if any(getattr(m, "bias_param", None) is not None for m in (self.dense_in, self.siglu_weight, self.dense_out)):
            return False
        if stash_active():
            return False
        wgu = adjacent_weights([self.dense_in.weight, self.siglu_weight.weight])
        x2 = x.reshape(-1, x.shape[-1])
        return (wgu is not None and nt_fused_mlp_enabled(x2, wgu) and bool(ext().gemm_nt_swiglu_ok(x2, wgu))
                and self.dense_out.weight.shape[1] % 256 == 0 and x.shape[-1] % 256 == 0)

    def _swiglu_bwd_wdt(self, x: torch.Tensor, z: torch.Tensor) -> Optional[torch.Tensor]:
        """The cached ``W_down^T`` when the SwiGLU + down projection run as ``_SwiGLUDown`` (GPU bf16 training, TP 1,
        bias-free, no GEMM-keeping checkpoint region, a shape the policy ``nt_swiglu_bwd_enabled`` picks), else None."""
        if not (use_native(z) and z.dtype == torch.bfloat16 and torch.is_grad_enabled() and z.requires_grad):
            return None
        if self.topology is not None and self.topology.config.model_parallel_size > 1:
            return None
        if self.dense_out.bias_param is not None or stash_active():
            return None
        wd = self.dense_out.weight
        x2 = x.reshape(-1, x.shape[-1])  # shaped like the output gradient dY [T, H]
        if x2.shape[1] != wd.shape[0] or not nt_swiglu_bwd_enabled(x2, (int(wd.shape[1]), int(wd.shape[0]))):
            return None
        wdt = _transposed([wd], wd)
        if wdt is None:  # weights under the cache's size floor: a per-call transpose
            wdt = transpose2d(wd.detach())
        return wdt if ext().gemm_nt_ok(x2, wdt) else None

    def forward(self, x: torch.Tensor, sp_shard: bool = False) -> torch.Tensor:
        """``sp_shard``: ``x`` is this rank's sequence-parallel token shard; its gather runs folded into (and overlapped
        with) the gate/up GEMM (``tp_overlap.sp_gather_column``)."""
        if sp_shard:
            mods = [self.dense_in, self.siglu_weight]
            z = sp_gather_column(x, [m.weight for m in mods], [m.bias_param for m in mods], self.topology)
            return self.dense_out.forward_sequence_parallel(swiglu_ops.swiglu_fused(z))
        if self._fused_eligible(x):
            return _SwiGLUMLPFused.apply(x.contiguous(), self.dense_in.weight, self.siglu_weight.weight,
                                         self.dense_out.weight)
        z = fused_column_linear(x, [self.dense_in, self.siglu_weight], self.topology)
        wdt = self._swiglu_bwd_wdt(x, z)
        if wdt is not None:
            return _SwiGLUDown.apply(z, self.dense_out.weight, wdt)
        h = swiglu_ops.swiglu_fused(z)
        if self.topology is not None and self.topology.config.sequence_parallel:
            return self.dense_out.forward_sequence_parallel(h)
        return self.dense_out(h)
