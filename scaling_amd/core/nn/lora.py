"""Parallel LoRA adapter (reference ``src/scaling/core/nn/lora.py:12-210``).

q/k/v adapters: Column(in->rank, gathered) -> Column(rank->out, parallel out, zero init);
dense adapter: Column(in->rank, parallel) -> Row(rank->out, parallel in).  ``get_delta_weights``
returns this rank's shard of ``scaling * B @ A`` for weight merging.
"""
from __future__ import annotations

from functools import partial
from typing import Optional, Union

import torch

from ..topology import Topology
from .linear import ColumnParallelLinear, RowParallelLinear
from .linear.utils import all_concat
from .lora_config import LoRAModuleType


class ParallelLoRa(torch.nn.Module):
    def __init__(
        self,
        in_features: int,
        out_features: int,
        lora_module_type: LoRAModuleType,
        rank: int,
        bias: bool = False,
        alpha: int = 1,
        dtype: torch.dtype = torch.float32,
        kaiming_a: Optional[float] = 1.0e-5,
        device: Optional[torch.device] = None,
        dropout: Optional[float] = None,
        topology: Optional[Topology] = None,
    ) -> None:
        super().__init__()
        assert rank <= in_features, f"LoRa Rank: {rank} is greater than the input dimensionality: {in_features}"
        self.scaling = alpha / rank
        self.topology = topology
        self.model_parallel_size = 1 if topology is None else topology.config.model_parallel_size
        if self.model_parallel_size > 1:
            assert rank % self.model_parallel_size == 0, "LoRA rank must be divisible by the model parallel size"
            assert out_features % self.model_parallel_size == 0, "out_features must be divisible by mp size"
        self.dropout = torch.nn.Dropout(dropout) if dropout is not None else None
        self.lora_module_type = lora_module_type
        init_a = partial(torch.nn.init.kaiming_uniform_, a=kaiming_a)
        kw = dict(bias=bias, device=device, dtype=dtype, topology=topology)
        self.dense_out: Union[ColumnParallelLinear, RowParallelLinear]
        if lora_module_type != LoRAModuleType.DENSE:
            self.dense_in = ColumnParallelLinear(in_features, rank, init_method=init_a, parallel_output=False, **kw)
            self.dense_out = ColumnParallelLinear(
                rank, out_features, init_method=torch.nn.init.zeros_, parallel_output=True, **kw
            )
        else:
            self.dense_in = ColumnParallelLinear(in_features, rank, init_method=init_a, parallel_output=True, **kw)
            self.dense_out = RowParallelLinear(
                rank, out_features, init_method=torch.nn.init.zeros_, parallel_input=True, parallel_output=False, **kw
            )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.dense_in(x)
        if self.dropout is not None:
            x = self.dropout(x)
        if getattr(self.dense_out, "bias", None) is None:  # scale the rank-wide intermediate, not the out-wide result (same math)
            return self.dense_out(x * self.scaling)
        return self.dense_out(x) * self.scaling

    def get_delta_weights(self) -> torch.Tensor:
        mp = self.model_parallel_size > 1
        dense = self.lora_module_type == LoRAModuleType.DENSE
        a = all_concat(self.dense_in.weight, dim=-2, topology=self.topology) if mp else self.dense_in.weight
        b = self.dense_out.weight
        if mp:
            b = all_concat(b, dim=-1 if dense else -2, topology=self.topology)
        delta = (b @ a) * self.scaling
        if mp:
            i = self.topology.model_parallel_rank if self.topology is not None else 0
            n = self.model_parallel_size
            if not dense:
                sz = delta.shape[0] // n
                delta = delta[i * sz : (i + 1) * sz]
            else:
                sz = delta.shape[1] // n
                delta = delta[:, i * sz : (i + 1) * sz]
        return delta
