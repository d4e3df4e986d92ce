"""TP (de)sharding of parameters for layout-independent checkpoints (reference ``utils/param_merge.py``).

``merge_parameter`` gathers all TP shards with ONE all-gather (instead of mp sequential broadcasts)
and concatenates along ``model_parallel_dimension`` on the host.
"""
from __future__ import annotations

from typing import Any

import torch
import torch.distributed as dist


def merge_parameter(parameter: torch.Tensor, core_parameter_meta: Any, topology: Any) -> torch.Tensor:
    if topology is None or topology.config.model_parallel_size == 1 or not core_parameter_meta.is_model_parallel:
        return parameter.detach().clone().cpu()
    mp = topology.config.model_parallel_size
    local = parameter.detach().contiguous()
    shards = [torch.empty_like(local) for _ in range(mp)]
    dist.all_gather(shards, local, group=topology.model_parallel_group)
    return torch.cat([s.cpu() for s in shards], dim=core_parameter_meta.model_parallel_dimension)


def split_parameter(parameter: torch.Tensor, core_parameter_meta: Any, topology: Any) -> torch.Tensor:
    mp = topology.config.model_parallel_size
    dim = core_parameter_meta.model_parallel_dimension
    assert dim is not None
    assert parameter.size(dim) % mp == 0, (
        f"cannot slice {core_parameter_meta.layer_class_name} {core_parameter_meta.parameter_name} of size "
        f"{parameter.size(dim)} in dimension {dim} by model parallel size {mp}"
    )
    n = parameter.size(dim) // mp
    return parameter.narrow(dim, topology.model_parallel_rank * n, n).contiguous()
