from __future__ import annotations

from enum import Enum
from typing import Optional, Union

import torch

from ...topology import Topology
from .layernorm import LayerNorm
from .layernorm_config import LayerNormConfig
from .rms_norm import RMSNorm


class NormType(Enum):
    LAYERNORM = "layernorm"
    RMS = "rms"


def get_norm(
    norm_type: NormType,
    layernorm_config: Optional[LayerNormConfig],
    dimensions: int,
    device: torch.device,
    dtype: torch.dtype,
    bitfit_bias_name: Optional[str] = None,
    topology: Optional[Topology] = None,
) -> Union[LayerNorm, RMSNorm]:
    assert layernorm_config is not None
    if norm_type == NormType.LAYERNORM:
        return LayerNorm(layernorm_config, dimensions, device, dtype, bitfit_bias_name, topology)
    if norm_type == NormType.RMS:
        return RMSNorm(dimensions, device, layernorm_config, dtype, topology)
    raise NotImplementedError(str(norm_type))
