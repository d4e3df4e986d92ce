"""Row-parallel linear: weight ``[out, in/tp]`` (reference ``row_parallel_linear.py:16-169``).

The (replicated) bias is added after the TP reduction, as in the reference.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ...topology import Topology
from ..parameter_meta import CoreParameterMeta
from .utils import all_reduce, all_reduce_scatter_to_sequence_parallel, all_shard, get_device
from .main_grad import linear as main_grad_linear
from .tp_overlap import chunked_supported, row_parallel_chunked


class RowParallelLinear(torch.nn.Module):
    def __init__(
        self,
        in_features: int,
        out_features: int,
        bias: bool = True,
        device: Optional[torch.device] = None,
        dtype: torch.dtype = torch.float32,
        topology: Optional[Topology] = None,
        init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
        parallel_input: bool = False,
        parallel_output: bool = False,
        bitfit_bias_name: Optional[str] = None,
    ) -> None:
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self._device = get_device(topology=topology, device=device)
        self.dtype = dtype
        self.topology = topology
        self.init_method = init_method
        self.parallel_input = parallel_input
        self.parallel_output = parallel_output
        self.model_parallel_size = 1 if topology is None else topology.config.model_parallel_size
        assert in_features % self.model_parallel_size == 0, (
            f"cannot row parallelize, in_features ({in_features}) "
            f"needs to be divisible by model parallel size ({self.model_parallel_size})"
        )
        self.input_features_per_partition = in_features // self.model_parallel_size
        self.weight = torch.nn.Parameter(
            torch.empty(out_features, self.input_features_per_partition, device=self._device, dtype=dtype)
        )
        init_method(self.weight)
        CoreParameterMeta.register_on_parameter(self.weight, is_model_parallel=True, model_parallel_dimension=1)
        self.bias_name: Optional[str] = None
        if bias:
            self.bias_name = "bias" if not bitfit_bias_name else f"bias_{bitfit_bias_name}"
            b = torch.nn.Parameter(torch.zeros(out_features, device=self._device, dtype=dtype))
            setattr(self, self.bias_name, b)
            CoreParameterMeta.register_on_parameter(b, is_model_parallel=False)

    @property
    def bias_param(self) -> Optional[torch.Tensor]:
        return getattr(self, self.bias_name) if self.bias_name is not None else None

    def _chunks(self) -> int:
        if self.topology is None or self.model_parallel_size == 1:
            return 1
        return int(getattr(self.topology.config, "tensor_parallel_comm_chunks", 1))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.parallel_input and self.topology is not None:
            x = all_shard(x, dim=-1, topology=self.topology)
        reduce = not self.parallel_output and self.topology is not None
        if reduce and chunked_supported(x, self.model_parallel_size, self._chunks(), False):
            out = row_parallel_chunked(x, self.weight, self.topology, False, self._chunks())
        else:
            out = main_grad_linear(x, self.weight)
            if reduce:
                out = all_reduce(out, topology=self.topology)
        b = self.bias_param
        return out if b is None else out + b

    def forward_sequence_parallel(self, x: torch.Tensor) -> torch.Tensor:
        """``reduce_scatter_to_sequence_parallel(self(x))`` for a ``parallel_output`` layer (attention dense / MLP
        dense_out under sequence parallelism), with the reduce-scatter overlapped piecewise with the GEMM when
        ``topology.tensor_parallel_comm_chunks > 1`` (bias-free layers; a bias keeps the reference's order)."""
        assert self.parallel_output and self.topology is not None
        if (self.parallel_input and self.bias_param is None
                and chunked_supported(x, self.model_parallel_size, self._chunks(), True)):
            return row_parallel_chunked(x, self.weight, self.topology, True, self._chunks())
        return all_reduce_scatter_to_sequence_parallel(self(x), self.topology)
