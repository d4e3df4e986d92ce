"""RMSNorm layer (reference ``src/scaling/core/nn/norm/rms_norm.py:21-61``) on the fused HIP kernel."""
from __future__ import annotations

from typing import Optional

import torch

from ....ops import norm as norm_ops
from ...topology import Topology
from ..linear.utils import gather_from_sequence_parallel_region
from ..parameter_meta import CoreParameterMeta
from .layernorm_config import LayerNormConfig


class RMSNorm(torch.nn.Module):
    def __init__(
        self,
        dimensions: int,
        device: torch.device,
        config: LayerNormConfig,
        dtype: torch.dtype = torch.float32,
        topology: Optional[Topology] = None,
    ) -> None:
        super().__init__()
        self.eps = config.layernorm_epsilon
        self.topology = topology
        self.config = config
        self.weight = torch.nn.Parameter(torch.ones(dimensions, dtype=dtype, device=device))
        CoreParameterMeta.register_on_parameter(self.weight, is_model_parallel=False)

    def _norm(self, x: torch.Tensor) -> torch.Tensor:
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.eps)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = norm_ops.rms_norm(x, self.weight, self.eps)
        if self.topology is not None and self.topology.config.sequence_parallel:
            out = gather_from_sequence_parallel_region(out, topology=self.topology, tensor_parallel_output_grad=True)
        return out

    def forward_add(self, x: torch.Tensor, res: Optional[torch.Tensor], gather: bool = True
                    ) -> tuple[torch.Tensor, torch.Tensor]:
        """``s = x + res; return s, self(s)`` with the residual add fused into the norm kernel (``res=None``: s = x,
        the gradient reaching s is added inside the norm backward).  ``gather=False``: under sequence parallelism the
        normalised output stays this rank's token shard (its consumer gathers it, ``tp_overlap.sp_gather_column``)."""
        s, out = norm_ops.add_rms_norm(x, res, self.weight, self.eps)
        if gather and self.topology is not None and self.topology.config.sequence_parallel:
            out = gather_from_sequence_parallel_region(out, topology=self.topology, tensor_parallel_output_grad=True)
        return s, out

    def gemv_prologue(self) -> Optional[tuple[torch.Tensor, float]]:
        """``(weight, eps)`` when this norm can run as the RMSNorm prologue of a decode GEMV (``ext().gemv_norm``):
        the normalised rows must be consumed locally, i.e. no sequence-parallel gather after the norm."""
        if self.topology is not None and self.topology.config.sequence_parallel:
            return None
        return self.weight, self.eps
