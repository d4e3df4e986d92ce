"""Lazy layer construction (reference ``parallel_module/layer_spec.py:8-30``)."""
from __future__ import annotations

from typing import Any, Optional, Type

import torch


class LayerSpec:
    def __init__(self, module_class: Type[torch.nn.Module], **kwargs: Any) -> None:
        self.module_class = module_class
        self.kwargs = kwargs

    def initialize(self, device: Optional[torch.device] = None) -> torch.nn.Module:
        module = self.module_class(**self.kwargs)
        if device is not None:
            module = module.to(device)
        elif torch.cuda.is_available():
            module = module.cuda()
        return module


class TiedLayerSpec(LayerSpec):
    def __init__(self, key: str, tied_weight_attributes: list[str], module_class: Type[torch.nn.Module], **kwargs: Any) -> None:
        super().__init__(module_class=module_class, **kwargs)
        self.key = key
        assert len(set(tied_weight_attributes)) == len(tied_weight_attributes), (
            f"duplicates in tied_weight_attributes: {tied_weight_attributes}"
        )
        self.tied_weight_attributes = tied_weight_attributes
