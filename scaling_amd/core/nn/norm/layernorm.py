"""LayerNorm layer (reference ``src/scaling/core/nn/norm/layernorm.py:14-85``) on the fused HIP kernel."""
from __future__ import annotations

from typing import Optional

import torch

from ....ops import norm as norm_ops
from ...topology import Topology
from ..linear.utils import gather_from_sequence_parallel_region
from ..parameter_meta import CoreParameterMeta
from .layernorm_config import LayerNormConfig


class LayerNorm(torch.nn.Module):
    def __init__(
        self,
        config: LayerNormConfig,
        normalized_shape: int,
        device: torch.device,
        dtype: torch.dtype = torch.float32,
        bitfit_bias_name: Optional[str] = None,
        topology: Optional[Topology] = None,
    ):
        super().__init__()
        self.config = config
        self.bias_name = "bias" if not bitfit_bias_name else f"bias_{bitfit_bias_name}"
        self.normalized_shape = torch.Size((normalized_shape,))
        self.topology = topology
        self.weight = torch.nn.Parameter(torch.ones(self.normalized_shape, device=device, dtype=dtype))
        CoreParameterMeta.register_on_parameter(self.weight, is_model_parallel=False)
        b = torch.nn.Parameter(torch.zeros(self.normalized_shape, device=device, dtype=dtype))
        setattr(self, self.bias_name, b)
        CoreParameterMeta.register_on_parameter(b, is_model_parallel=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = norm_ops.layer_norm(x, self.weight, getattr(self, self.bias_name), self.config.layernorm_epsilon)
        if self.topology is not None and self.topology.config.sequence_parallel:
            out = gather_from_sequence_parallel_region(out, topology=self.topology, tensor_parallel_output_grad=True)
        return out

    def forward_add(self, x: torch.Tensor, res: Optional[torch.Tensor], gather: bool = True
                    ) -> tuple[torch.Tensor, torch.Tensor]:
        """``s = x + res; return s, self(s)`` with the residual add fused into the norm kernel (``res=None``: s = x,
        the gradient reaching s is added inside the norm backward).  ``gather=False``: under sequence parallelism the
        normalised output stays this rank's token shard (its consumer gathers it, ``tp_overlap.sp_gather_column``)."""
        s, out = norm_ops.add_layer_norm(x, res, self.weight, getattr(self, self.bias_name), self.config.layernorm_epsilon)
        if gather and self.topology is not None and self.topology.config.sequence_parallel:
            out = gather_from_sequence_parallel_region(out, topology=self.topology, tensor_parallel_output_grad=True)
        return s, out
