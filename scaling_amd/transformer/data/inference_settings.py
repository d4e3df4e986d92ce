"""Inference-time settings carried through the layers (reference ``data/inference_settings.py``)."""
from __future__ import annotations

from typing import NamedTuple, Optional, Union

from pydantic import Field

from ...core import BaseConfig


class Control(BaseConfig):
    token_index: int = Field(description="token index to be controlled")
    factor: float = Field(description="control factor")


class InferenceSuppressionParameters(NamedTuple):
    contextual_control_threshold: Optional[float]
    control_log_additive: bool
    controls: Optional[list[Control]]


class InferenceSettings:
    def __init__(self, use_cache: bool, reset_cache: bool, cache_index: int, embedding_layers: list[int],
                 input_image_locations: Optional[list[tuple[int, int, int]]] = None,
                 inference_control_parameters: Optional[list[InferenceSuppressionParameters]] = None) -> None:
        self.use_cache = use_cache
        self.reset_cache = reset_cache
        self.cache_index = cache_index
        self.embedding_layers = embedding_layers
        self.input_image_locations = input_image_locations
        self.inference_control_parameters = inference_control_parameters
        self.control_log_additive_batch: Union[bool, list[bool]]
        flags = [p.control_log_additive for p in (inference_control_parameters or [])]
        if not flags or all(flags):
            self.control_log_additive_batch = True
        elif not any(flags):
            self.control_log_additive_batch = False
        else:
            self.control_log_additive_batch = flags
