"""Tensor-parallel MLPs (reference ``src/scaling/core/nn/mlp.py:21-167``).

``ParallelSwiGLUMLP`` keeps the reference parameters (``dense_in``, ``siglu_weight``, ``dense_out``)
but runs ``dense_in``/``siglu_weight`` as one fused GEMM whose ``[..., 2F]`` output feeds the HIP
SwiGLU kernel directly (and whose backward receives the fused gradient from that kernel).

The forward / input-gradient GEMMs are plain library GEMMs (hipBLASLt).  Rounds 3-5 built a hand-written NT GEMM with
the SwiGLU forward / backward in its epilogues; it stayed 1-6 % behind hipBLASLt per shape and lost in the 7B step
even with the fused epilogues (profiles/gemm_nt_round_remap_ab_r5.log, profiles/swiglu_bwd_nt_ab_r5.log), so it was
deleted in round 6 (git history before "Delete the NT GEMM").
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ...ops import swiglu as swiglu_ops
from ...ops._ext import ext, use_native
from ..topology import Topology
from .activation_function import ActivationFunction, get_activation_function
from .linear import ColumnParallelLinear, RowParallelLinear
from .linear.fused import fused_column_linear
from .linear.tp_overlap import sp_gather_column
from .linear.main_grad import adjacent_weights


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

    def forward(self, x: torch.Tensor, sp_shard: bool = False) -> torch.Tensor:
        """``sp_shard``: ``x`` is this rank's sequence-parallel token shard; its gather runs folded into (and overlapped
        with) the gate/up GEMM (``tp_overlap.sp_gather_column``)."""
        if sp_shard:
            mods = [self.dense_in, self.siglu_weight]
            z = sp_gather_column(x, [m.weight for m in mods], [m.bias_param for m in mods], self.topology)
            return self.dense_out.forward_sequence_parallel(swiglu_ops.swiglu_fused(z))
        z = fused_column_linear(x, [self.dense_in, self.siglu_weight], self.topology)
        h = swiglu_ops.swiglu_fused(z)
        if self.topology is not None and self.topology.config.sequence_parallel:
            return self.dense_out.forward_sequence_parallel(h)
        return self.dense_out(h)
