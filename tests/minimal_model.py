"""Minimal pipeline model for engine tests (role of the reference's ``tests/core/minimal``):
embedding -> column-parallel linear -> row-parallel linear -> layernorm / tied embedding head."""
from __future__ import annotations

from typing import Any, Optional

import torch

from scaling_amd.core import (
    BaseDatasetBatch,
    BaseLayer,
    BaseLayerIO,
    ColumnParallelLinear,
    LayerNorm,
    LayerNormConfig,
    LayerSpec,
    RowParallelLinear,
    TiedLayerSpec,
    Topology,
    VocabParallelEmbedding,
)

VOCAB, HIDDEN = 16, 8


class MinimalBatch(BaseDatasetBatch):
    def __init__(self, inputs: Optional[torch.Tensor] = None, targets: Optional[torch.Tensor] = None):
        self.inputs = inputs
        self.targets = targets

    def only_inputs(self) -> "MinimalBatch":
        return MinimalBatch(inputs=self.inputs)

    def only_targets(self) -> "MinimalBatch":
        return MinimalBatch(targets=self.targets)

    def to_(self, device: torch.device) -> None:
        for n in ("inputs", "targets"):
            t = getattr(self, n)
            if t is not None:
                setattr(self, n, t.to(device))


class MinimalIO(BaseLayerIO):
    def __init__(self, activations: torch.Tensor):
        self.activations = activations


class _Base(BaseLayer[Any, MinimalIO, MinimalIO]):
    @staticmethod
    def input_to_tuple(input: Any) -> tuple[Any, ...]:
        return (input.activations,) if isinstance(input, MinimalIO) else (input.inputs,)

    @staticmethod
    def tuple_to_input(d: tuple[Any, ...]) -> Any:
        return MinimalIO(activations=d[0])

    @staticmethod
    def output_to_tuple(output: MinimalIO) -> tuple[Any, ...]:
        return (output.activations,)

    @staticmethod
    def tuple_to_last_stage_activation(d: tuple[Any, ...]) -> MinimalIO:
        return MinimalIO(activations=d[0])


class MinimalEmbeddingInput(_Base):
    def __init__(self, topology: Optional[Topology] = None, device: Optional[torch.device] = None):
        super().__init__()
        self.embedding = VocabParallelEmbedding(VOCAB, HIDDEN, finetunable_token_ids=[], topology=topology,
                                                device=None if topology is not None else device)

    def forward(self, x: Any) -> MinimalIO:
        return MinimalIO(self.embedding(x.inputs))


class MinimalLinearColumnParallel(_Base):
    def __init__(self, topology: Optional[Topology] = None, device: Optional[torch.device] = None):
        super().__init__()
        self.linear = ColumnParallelLinear(HIDDEN, 2 * HIDDEN, topology=topology, parallel_output=True,
                                           device=None if topology is not None else device)

    def forward(self, x: MinimalIO) -> MinimalIO:
        return MinimalIO(torch.relu(self.linear(x.activations)))


class MinimalLinearRowParallel(_Base):
    def __init__(self, topology: Optional[Topology] = None, device: Optional[torch.device] = None):
        super().__init__()
        self.linear = RowParallelLinear(2 * HIDDEN, HIDDEN, topology=topology, parallel_input=True,
                                        device=None if topology is not None else device)

    def forward(self, x: MinimalIO) -> MinimalIO:
        return MinimalIO(self.linear(x.activations))


class MinimalLayerNorm(_Base):
    def __init__(self, topology: Optional[Topology] = None, device: Optional[torch.device] = None):
        super().__init__()
        dev = topology.device if topology is not None else (device or torch.device("cpu"))
        self.norm = LayerNorm(LayerNormConfig(), HIDDEN, device=dev, topology=topology)

    def forward(self, x: MinimalIO) -> MinimalIO:
        return MinimalIO(self.norm(x.activations))


class MinimalEmbeddingTied(MinimalEmbeddingInput):
    def forward(self, x: MinimalIO) -> MinimalIO:  # type: ignore[override]
        return MinimalIO(torch.nn.functional.linear(x.activations, self.embedding.weight))


def layer_specs(weight_tying: bool, topology: Optional[Topology] = None) -> list[LayerSpec]:
    kw = {} if topology is None else {"topology": topology}
    if weight_tying:
        return [
            TiedLayerSpec(module_class=MinimalEmbeddingInput, key="embedding_tying",
                          tied_weight_attributes=["embedding.weight"], **kw),
            LayerSpec(MinimalLinearColumnParallel, **kw),
            LayerSpec(MinimalLinearRowParallel, **kw),
            TiedLayerSpec(module_class=MinimalEmbeddingTied, key="embedding_tying",
                          tied_weight_attributes=["embedding.weight"], **kw),
        ]
    return [LayerSpec(MinimalEmbeddingInput, **kw), LayerSpec(MinimalLinearColumnParallel, **kw),
            LayerSpec(MinimalLinearRowParallel, **kw), LayerSpec(MinimalLayerNorm, **kw)]
