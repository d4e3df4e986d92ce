"""Tied weights across pipeline stages (reference ``parallel_module/tied_layer_index.py:11-224``).

For every tied key: which pipe ranks hold a copy, a process group per (dp, mp) over those ranks for
the grad all-reduce / init broadcast, and within a stage all duplicate modules alias the local main
module's weights.
"""
from __future__ import annotations

import collections
from typing import Any, Optional

import torch
import torch.distributed as dist

from .layer_spec import LayerSpec, TiedLayerSpec
from .pipeline_partitioning import PipePartitionCoordinates


class TiedLayerInformation:
    def __init__(self) -> None:
        self.is_local = False
        self.layer_indices: set[int] = set()
        self.pipe_parallel_ranks: set[int] = set()
        self.tied_weight_attributes: set[str] = set()
        self.process_group: Any = None
        self.global_ranks: Optional[list[int]] = None

    def add(self, layer_index: int, pipe_parallel_rank: int, is_local: bool, tied_weight_attributes: list[str]) -> None:
        self.layer_indices.add(layer_index)
        self.pipe_parallel_ranks.add(pipe_parallel_rank)
        self.is_local = self.is_local or is_local
        self.tied_weight_attributes.update(tied_weight_attributes)

    def build_process_groups(self, topology: Any) -> None:
        for dp in range(topology.config.data_parallel_size):
            for mp in range(topology.config.model_parallel_size):
                ranks = sorted(
                    topology.get_global_rank(data_parallel_rank=dp, model_parallel_rank=mp, pipe_parallel_rank=pp)
                    for pp in self.pipe_parallel_ranks
                )
                group = dist.new_group(ranks) if len(ranks) > 1 and topology.is_distributed_initialized else None
                if topology.config.global_rank in ranks:
                    self.process_group, self.global_ranks = group, ranks


class TiedModule:
    def __init__(self, module: torch.nn.Module, is_main: bool, is_local_main: bool, tied_weight_attributes: list[str]):
        self.module = module
        self.is_main = is_main
        self.is_local_main = is_local_main
        self.tied_weight_attributes = set(tied_weight_attributes)


def _resolve(module: torch.nn.Module, dotted: str) -> tuple[torch.nn.Module, str]:
    parts = dotted.split(".")
    for p in parts[:-1]:
        module = getattr(module, p)
    return module, parts[-1]


class TiedLayerIndex:
    def __init__(self, pipe_partition_coordinates: list[PipePartitionCoordinates], layer_specs: list[LayerSpec],
                 topology: Any, device: Optional[torch.device] = None) -> None:
        own = pipe_partition_coordinates[topology.pipe_parallel_rank]
        self.layer_index_to_pipe_parallel_rank = {
            li: pr for pr, c in enumerate(pipe_partition_coordinates) for li in range(c.start, c.end)
        }
        self.tied_information_by_key: dict[str, TiedLayerInformation] = collections.defaultdict(TiedLayerInformation)
        for li, spec in enumerate(layer_specs):
            if isinstance(spec, TiedLayerSpec):
                self.tied_information_by_key[spec.key].add(
                    li, self.layer_index_to_pipe_parallel_rank[li], own.start <= li < own.end, spec.tied_weight_attributes
                )
        for key in sorted(self.tied_information_by_key):
            self.tied_information_by_key[key].build_process_groups(topology)
        seen: collections.Counter = collections.Counter()
        seen_local: collections.Counter = collections.Counter()
        self.tied_modules_local_main_by_key: dict[str, TiedModule] = {}
        self.tied_parameters_by_key: dict[str, dict[str, torch.nn.Parameter]] = {}
        self.tied_modules_by_layer_index: dict[int, TiedModule] = {}
        for li, spec in enumerate(layer_specs):
            if not isinstance(spec, TiedLayerSpec):
                continue
            is_local = own.start <= li < own.end
            is_main = seen[spec.key] == 0
            is_local_main = seen_local[spec.key] == 0
            seen[spec.key] += 1
            if not is_local:
                continue
            seen_local[spec.key] += 1
            module = spec.initialize(device=device if device is not None else getattr(topology, "_device", None))
            tm = TiedModule(module, is_main, is_local_main, spec.tied_weight_attributes)
            if is_local_main:
                self.tied_modules_local_main_by_key[spec.key] = tm
                attrs = self.tied_information_by_key[spec.key].tied_weight_attributes
                self.tied_parameters_by_key[spec.key] = {n: p for n, p in module.named_parameters() if n in attrs}
            else:
                main = self.tied_modules_local_main_by_key[spec.key].module
                for attr in spec.tied_weight_attributes:
                    m_main, name = _resolve(main, attr)
                    m_dup, _ = _resolve(module, attr)
                    setattr(m_dup, name, getattr(m_main, name))
            self.tied_modules_by_layer_index[li] = tm

    def get_module_by_layer_index(self, layer_index: int) -> torch.nn.Module:
        return self.tied_modules_by_layer_index[layer_index].module

    def get_tied_weight_attributes_by_layer_index(self, layer_index: int) -> set[str]:
        return self.tied_modules_by_layer_index[layer_index].tied_weight_attributes

    def local_parameters_and_process_groups(self) -> list[tuple[torch.nn.Parameter, Any, set[int]]]:
        out = []
        for key in sorted(self.tied_parameters_by_key):
            for name in sorted(self.tied_parameters_by_key[key]):
                info = self.tied_information_by_key[key]
                if len(info.pipe_parallel_ranks) > 1:
                    assert info.process_group is not None or not dist.is_initialized()
                out.append((self.tied_parameters_by_key[key][name], info.process_group, info.pipe_parallel_ranks))
        return out

    def layer_index_is_tied_global_duplicate(self, layer_index: int) -> bool:
        tm = self.tied_modules_by_layer_index.get(layer_index)
        return tm is not None and not tm.is_main

    def layer_index_is_tied_local_duplicate(self, layer_index: int) -> bool:
        tm = self.tied_modules_by_layer_index.get(layer_index)
        return tm is not None and not tm.is_local_main

    def layer_index_to_tied_local_duplicate_parameter_names(self, layer_index: int) -> set[str]:
        tm = self.tied_modules_by_layer_index.get(layer_index)
        if tm is None or tm.is_local_main:
            return set()
        return tm.tied_weight_attributes
