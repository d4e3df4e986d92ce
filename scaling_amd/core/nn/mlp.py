"""Tensor-parallel MLPs (reference ``src/scaling/core/nn/mlp.py:21-167``).

``ParallelSwiGLUMLP`` keeps the reference parameters (``dense_in``, ``siglu_weight``, ``dense_out``)
but runs ``dense_in``/``siglu_weight`` as one fused GEMM whose ``[..., 2F]`` output feeds the HIP
SwiGLU kernel directly (and whose backward receives the fused gradient from that kernel).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ...ops import swiglu as swiglu_ops
from ..topology import Topology
from .activation_function import ActivationFunction, get_activation_function
from .linear import ColumnParallelLinear, RowParallelLinear
from .linear.fused import fused_column_linear


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

    def forward(self, x: torch.Tensor) -> torch.Tensor:
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

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        z = fused_column_linear(x, [self.dense_in, self.siglu_weight], self.topology)
        h = swiglu_ops.swiglu_fused(z)
        if self.topology is not None and self.topology.config.sequence_parallel:
            return self.dense_out.forward_sequence_parallel(h)
        return self.dense_out(h)
