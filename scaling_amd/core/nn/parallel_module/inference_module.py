"""Single-process multi-GPU inference module (reference ``parallel_module/inference_module.py``).

Layers are split over a device list; the layer IO hops devices at stage boundaries (``to_`` with
non-blocking copies over xGMI peer access).  ``HiddenStateRecorder`` captures sub-module outputs.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import partial
from typing import Any, Optional, Sequence

import torch

from ...data import BaseLayerIO
from ...topology import PipePartitionMethod
from .layer_spec import LayerSpec, TiedLayerSpec
from .partitioned_module import PipePartitionedModule


@dataclass
class RecorderSetting:
    include_modules: Optional[Sequence[str]] = ("",)
    exclude_modules: Optional[Sequence[str]] = None

    def __post_init__(self) -> None:
        assert self.include_modules is None or self.exclude_modules is None, (
            "Cannot specify both include_modules and exclude_modules"
        )


class HiddenStateRecorder:
    def __init__(self, module: PipePartitionedModule, recorder_settings_per_layer: dict[int, RecorderSetting]):
        self._module = module
        self.recorder_settings_per_layer = recorder_settings_per_layer
        self.current_record: dict[int, dict[str, Any]] = {k: {} for k in recorder_settings_per_layer}
        self._hooks: list[Any] = []

    def __enter__(self) -> None:
        self.start_recording()

    def __exit__(self, *_args: Any) -> None:
        self.stop_recording()

    def record_output(self, module: torch.nn.Module, input: Any, output: Any, layer_index: int, name: str) -> None:
        self.current_record[layer_index][name] = output

    def start_recording(self) -> None:
        for li, s in self.recorder_settings_per_layer.items():
            if s.include_modules is None and s.exclude_modules is None:
                continue  # neither list given: nothing is recorded for this layer (reference semantics)
            layer = self._module._layers[li]
            for name, sub in layer.named_modules():
                take = (name in s.include_modules) if s.include_modules is not None else (name not in s.exclude_modules)
                if take:
                    self._hooks.append(sub.register_forward_hook(partial(self.record_output, layer_index=li, name=name)))

    def stop_recording(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def delete_records(self) -> None:
        self.current_record = {k: {} for k in self.recorder_settings_per_layer}


class InferenceModule(PipePartitionedModule):
    def __init__(self, layer_specs: list[LayerSpec], devices: Sequence[Any] = (0,),
                 pipe_partition_method: PipePartitionMethod = PipePartitionMethod.UNIFORM,
                 pipe_partition_overwrite: Optional[list[int]] = None):
        specs = [LayerSpec(s.module_class, **s.kwargs) if isinstance(s, TiedLayerSpec) else s for s in layer_specs]
        super().__init__(layer_specs=specs, devices=devices, pipe_partition_method=pipe_partition_method,
                         pipe_partition_overwrite=pipe_partition_overwrite)
        self.eval()

    @torch.no_grad()
    def forward(self, x: BaseLayerIO) -> BaseLayerIO:
        assert self.devices is not None
        for device, c in zip(self.devices, self._pipe_partition_coordinates):
            for i, layer in enumerate(self._layers[c.start : c.end]):
                if i == 0:
                    x.to_(device)
                x = layer(x)
        return x

    @torch.no_grad()
    def forward_with_hidden_state_recorder(self, x: BaseLayerIO, recorder_settings_per_layer: Optional[dict[int, RecorderSetting]] = None):
        rec = HiddenStateRecorder(self, recorder_settings_per_layer or {})
        with rec:
            x = self.forward(x)
        return x, rec.current_record
