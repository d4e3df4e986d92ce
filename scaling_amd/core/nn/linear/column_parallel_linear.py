"""Column-parallel linear: weight ``[out/tp, in]`` (reference ``column_parallel_linear.py:23-159``)."""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ...topology import Topology
from ..parameter_meta import CoreParameterMeta
from .utils import all_concat, get_device, tp_input_grad_group
from .main_grad import linear as main_grad_linear


class ColumnParallelLinear(torch.nn.Module):
    def __init__(
        self,
        in_features: int,
        out_features: int,
        bias: bool = True,
        device: Optional[torch.device] = None,
        dtype: torch.dtype = torch.float32,
        topology: Optional[Topology] = None,
        init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
        parallel_output: bool = False,
        bitfit_bias_name: Optional[str] = None,
    ):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self._device = get_device(topology=topology, device=device)
        self.dtype = dtype
        self.topology = topology
        self.init_method = init_method
        self.parallel_output = parallel_output
        self.model_parallel_size = 1 if topology is None else topology.config.model_parallel_size
        assert out_features % self.model_parallel_size == 0, (
            f"cannot column parallelize, out_features ({out_features}) "
            f"needs to be divisible by model parallel size ({self.model_parallel_size})"
        )
        self.output_features_per_partition = out_features // self.model_parallel_size
        self.weight = torch.nn.Parameter(
            torch.empty(self.output_features_per_partition, in_features, device=self._device, dtype=dtype)
        )
        init_method(self.weight)
        CoreParameterMeta.register_on_parameter(self.weight, is_model_parallel=True, model_parallel_dimension=0)
        self.bias_name: Optional[str] = None
        if bias:
            self.bias_name = "bias" if not bitfit_bias_name else f"bias_{bitfit_bias_name}"
            b = torch.nn.Parameter(torch.zeros(self.output_features_per_partition, device=self._device, dtype=dtype))
            setattr(self, self.bias_name, b)
            CoreParameterMeta.register_on_parameter(b, is_model_parallel=True, model_parallel_dimension=0)

    @property
    def bias_param(self) -> Optional[torch.Tensor]:
        return getattr(self, self.bias_name) if self.bias_name is not None else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # copy_to region folded into the linear: its input-gradient all-reduce overlaps the wgrad GEMM
        out = main_grad_linear(x, self.weight, self.bias_param, tp_group=tp_input_grad_group(self.topology))
        if self.parallel_output or self.topology is None:
            return out
        return all_concat(out, dim=-1, topology=self.topology)
