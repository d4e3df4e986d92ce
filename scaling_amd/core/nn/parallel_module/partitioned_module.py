"""Pipeline-partitioned module with layout-independent per-layer checkpoints.

Parity: reference ``parallel_module/partitioned_module.py:35-371``: one file per global layer
``model_state_layer_{idx}_{ClassName}[_{sep}].pt`` holding TP-merged CPU tensors (written by
dp-rank 0 / mp-rank 0), glob-loading across several directories, optional bias cloning, TP split on
load, regex ignore/allowed-missing/allowed-unexpected key filters.  Works with a topology (one
process per GPU) or with a device list (single-process multi-GPU inference).
"""
from __future__ import annotations

import re
from pathlib import Path
from typing import Any, Optional, Sequence, Union

import torch

from ...logging import logger
from ...topology import PipePartitionMethod
from ...utils.checkpoint_writer import save_file
from ...utils.param_merge import merge_parameter, split_parameter
from ..linear.main_grad import invalidate_transposed_weights
from ..parameter_meta import CoreParameterMeta
from .layer_spec import LayerSpec, TiedLayerSpec
from .pipeline_partitioning import (
    PipePartitionCoordinates,
    pipe_partition_balanced,
    pipe_partition_from_indices,
    pipe_partition_uniform,
)
from .tied_layer_index import TiedLayerIndex


def key_match(key: str, list_of_patterns: list[str]) -> bool:
    return any(re.search(p, key) is not None for p in list_of_patterns)


def _load_state(f: Path) -> dict:
    # checkpoint files written by this framework: plain tensors only
    return torch.load(str(f), map_location="cpu", weights_only=True)


class PipePartitionedModule(torch.nn.Module):
    def __init__(
        self,
        layer_specs: list[LayerSpec],
        devices: Optional[Sequence[Any]] = None,
        topology: Any = None,
        pipe_partition_method: Optional[PipePartitionMethod] = None,
        pipe_partition_overwrite: Optional[list[int]] = None,
    ):
        super().__init__()
        assert (devices is None) ^ (topology is None), "Exactly either one of 'devices' or 'topology' must be specified"
        self.topology = topology
        self.devices: Optional[list[torch.device]] = None
        if devices is not None:
            self.devices = [
                d if isinstance(d, torch.device) else torch.device(d) if isinstance(d, str)
                else (torch.device("cuda", d) if torch.cuda.is_available() else torch.device("cpu"))
                for d in devices
            ]
        self._layer_specs = layer_specs
        if topology is None:
            self.pipe_partition_method = pipe_partition_method or PipePartitionMethod.UNIFORM
            self.pipe_partition_overwrite = pipe_partition_overwrite
        else:
            assert pipe_partition_method is None and pipe_partition_overwrite is None, (
                "pipe partitioning is configured through the topology"
            )
            self.pipe_partition_method = topology.config.pipe_partition_method
            self.pipe_partition_overwrite = topology.config.pipe_partition_overwrite
        self._initialize_layers()

    def _get_pipe_partition_coordinates(self) -> list[PipePartitionCoordinates]:
        n = len(self.devices) if self.devices is not None else self.topology.config.pipe_parallel_size
        if len(self._layer_specs) < n:
            raise RuntimeError(f"Number of layers ({len(self._layer_specs)}) is smaller than number of pipe partitions {n}")
        if self.pipe_partition_overwrite is not None:
            return pipe_partition_from_indices(self.pipe_partition_overwrite, num_layers=len(self._layer_specs))
        if self.pipe_partition_method == PipePartitionMethod.UNIFORM:
            return pipe_partition_uniform(len(self._layer_specs), n)
        if self.pipe_partition_method == PipePartitionMethod.BALANCED:
            return pipe_partition_balanced(self._layer_specs, n)
        raise NotImplementedError(f"Pipe partition method not known: {self.pipe_partition_method}")

    def _initialize_layers(self) -> None:
        coords = self._get_pipe_partition_coordinates()
        for idx, c in enumerate(coords):
            assert c.start < c.end, f"no parallel module layer spec assigned to index {idx}"
            if self.topology is None or self.topology.config.global_rank == 0:
                logger.info(f"pipe_parallel_rank {idx} gets layers {c.start}:{c.end}")
        self._all_pipe_partition_coordinates = coords
        self._pipe_partition_coordinates = coords if self.topology is None else [coords[self.topology.pipe_parallel_rank]]
        self.tied_layer_index: Optional[TiedLayerIndex] = None
        if self.topology is not None:
            self.tied_layer_index = TiedLayerIndex(coords, self._layer_specs, self.topology, device=self.topology.device)
        devices = self.devices if self.devices is not None else [self.topology.device]
        self._layers = torch.nn.ModuleList()
        self._layer_devices: list[torch.device] = []
        for device, c in zip(devices, self._pipe_partition_coordinates):
            for li in range(c.start, c.end):
                spec = self._layer_specs[li]
                if isinstance(spec, TiedLayerSpec) and self.tied_layer_index is not None:
                    layer = self.tied_layer_index.get_module_by_layer_index(li)
                    tied_attrs = self.tied_layer_index.get_tied_weight_attributes_by_layer_index(li)
                    is_tied = True
                else:
                    layer = spec.initialize(device=device)
                    tied_attrs, is_tied = set(), False
                for name, p in list(layer.named_parameters()) + list(layer.named_buffers()):
                    p_tied = is_tied and name in tied_attrs
                    if hasattr(p, "core_parameter_meta"):
                        p.core_parameter_meta.set(li, name, layer.__class__.__name__, p_tied)
                    else:
                        CoreParameterMeta.register_on_parameter(
                            p, is_model_parallel=False, layer_index=li, parameter_name=name,
                            layer_class_name=layer.__class__.__name__, is_tied=p_tied,
                        )
                self._layers.append(layer)
                self._layer_devices.append(device)
            # the last layer of a pipeline stage that feeds another stage hands its output to pipe p2p: layers that can
            # leave part of their output pending (TransformerLayerIO.residual_branch) resolve it there, so a stage
            # boundary moves (and a checkpoint saves) one tensor, not two
            if c.end > c.start and c.end < len(self._layer_specs) and hasattr(self._layers[-1], "set_stage_output"):
                self._layers[-1].set_stage_output(True)

    def _global_layer_indices(self) -> list[int]:
        return [li for c in self._pipe_partition_coordinates for li in range(c.start, c.end)]

    # ------------------------------------------------------------------ checkpoint
    def save_checkpoint(self, dir_: Union[Path, str], separate_file_for_parameters: Optional[list[str]] = None) -> None:
        opt = getattr(self, "_param_sync_optimizer", None)
        if opt is not None:  # parameters may still be in flight (async ZeRO all-gather)
            opt.wait_param_sync()
        if self.topology is not None and self.topology.data_parallel_rank != 0:
            return
        dir_ = Path(dir_)
        for li, layer in zip(self._global_layer_indices(), self._layers):
            states: dict[str, dict[str, torch.Tensor]] = {"": {}}
            for sep in separate_file_for_parameters or []:
                states[sep] = {}
            persistent = set(layer.state_dict().keys())
            for name, p in list(layer.named_parameters()) + list(layer.named_buffers()):
                if name not in persistent:
                    continue
                merged = merge_parameter(p, p.core_parameter_meta, self.topology) if self.topology is not None else p.detach().clone().cpu()
                target = ""
                for sep in separate_file_for_parameters or []:
                    if sep in name:
                        target = sep
                states[target][name] = merged
            if self.topology is None or self.topology.model_parallel_rank == 0:
                for sep, sd in states.items():
                    if not sd:
                        continue
                    fname = f"model_state_layer_{li}_{layer.__class__.__name__}{'' if sep == '' else '_'}{sep}.pt"
                    save_file(sd, dir_ / fname)

    def load_checkpoint(
        self,
        dir_: Union[Path, str, Sequence[Union[Path, str]]],
        add_bias_names_if_not_exist: Optional[list[str]] = None,
        add_bias_names_if_not_exist_exceptions: Optional[list[str]] = None,
        allowed_missing_keys_in_checkpoint: Optional[list[str]] = None,
        allowed_unexpected_keys_in_checkpoint: Optional[list[str]] = None,
        ignore_keys_in_checkpoint: Optional[list[str]] = None,
    ) -> None:
        paths = [Path(p) for p in (dir_ if isinstance(dir_, (list, tuple)) else [dir_])]
        missing_dirs = [p for p in paths if not p.is_dir()]
        if missing_dirs:
            raise RuntimeError(f"Weight set directories missing: {missing_dirs}")
        ignore = list(ignore_keys_in_checkpoint or [])
        # an ignored key keeps its initialisation: it is neither unexpected nor missing (the reference
        # removes it from the file dict but would then report it missing)
        allowed_missing = list(allowed_missing_keys_in_checkpoint or []) + ignore
        allowed_unexpected = list(allowed_unexpected_keys_in_checkpoint or []) + ignore
        missing, unexpected = set(), set()
        for li, layer in zip(self._global_layer_indices(), self._layers):
            sd: dict[str, torch.Tensor] = {}
            for p in paths:
                for f in sorted(p.glob(f"model_state_layer_{li}_{layer.__class__.__name__}*.pt")):
                    sd.update(_load_state(f))
            if add_bias_names_if_not_exist:
                for k in list(sd.keys()):
                    if add_bias_names_if_not_exist_exceptions and any(
                        part == e for part in k.split(".") for e in add_bias_names_if_not_exist_exceptions
                    ):
                        continue
                    if k.endswith(".bias"):
                        for bn in add_bias_names_if_not_exist:
                            if bn and (k + "_" + bn) not in sd:
                                sd[k + "_" + bn] = sd[k].clone()
            if self.topology is not None and self.topology.config.model_parallel_size > 1:
                for name, p in list(layer.named_parameters()) + list(layer.named_buffers()):
                    if name in sd and p.core_parameter_meta.is_model_parallel:
                        sd[name] = split_parameter(sd[name], p.core_parameter_meta, self.topology)
            for k in list(sd.keys()):
                if key_match(k, ignore):
                    del sd[k]
            res = layer.load_state_dict(sd, strict=False)
            missing.update(res.missing_keys)
            unexpected.update(res.unexpected_keys)
        invalidate_transposed_weights()
        bad_unexpected = {k for k in unexpected if not key_match(k, allowed_unexpected)}
        if unexpected - bad_unexpected:
            logger.warning(f"Ignoring unexpected keys in checkpoint: {unexpected - bad_unexpected}")
        if bad_unexpected:
            raise RuntimeError(f"Unexpected keys in checkpoint: {bad_unexpected}. You may add keys to 'allowed_unexpected_keys_in_checkpoint'.")
        bad_missing = {k for k in missing if not key_match(k, allowed_missing)}
        if missing - bad_missing:
            logger.warning(f"Ignoring missing keys in checkpoint: {missing - bad_missing}")
        if bad_missing:
            raise RuntimeError(f"Missing keys in checkpoint: {bad_missing}. You may add keys to 'allowed_missing_keys_in_checkpoint'.")
