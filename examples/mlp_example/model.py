"""3D-parallel MLP: alternating Column / Row parallel linears (reference ``examples/mlp_example/model.py``)."""
from __future__ import annotations

from typing import Any, Callable, Union

import torch
import torch.nn.functional as F

from scaling_amd.core import (
    BaseLayer,
    BaseLayerIO,
    BaseOptimizer,
    ColumnParallelLinear,
    LayerSpec,
    Optimizer,
    OptimizerParamGroup,
    OptimizerParamGroupConfig,
    ParallelModule,
    RowParallelLinear,
    Topology,
)

from .context import MLPContext
from .data import MNISTDatasetBatch


class MLPLayerIO(BaseLayerIO):
    def __init__(self, activations: torch.Tensor):
        self.activations = activations


class MLPBaseLayer(BaseLayer[MLPLayerIO, MLPLayerIO, MLPLayerIO]):
    @staticmethod
    def input_to_tuple(input: MLPLayerIO) -> tuple[Any, ...]:
        return (input.activations,)

    @staticmethod
    def tuple_to_input(d: tuple[Any, ...]) -> MLPLayerIO:
        return MLPLayerIO(activations=d[0])

    @staticmethod
    def output_to_tuple(output: MLPLayerIO) -> tuple[Any, ...]:
        return (output.activations,)

    @staticmethod
    def tuple_to_last_stage_activation(d: tuple[Any, ...]) -> MLPLayerIO:
        return MLPLayerIO(activations=d[0])


def _inputs(x: Union[MLPLayerIO, MNISTDatasetBatch]) -> torch.Tensor:
    t = x.activations if isinstance(x, MLPLayerIO) else x.inputs
    assert t is not None
    return torch.flatten(t, start_dim=1)


class MLPLinearColumnParallel(MLPBaseLayer):
    def __init__(self, in_features: int, out_features: int, topology: Topology, parallel_output: bool = True,
                 act_fn: Callable = lambda x: x, dtype: torch.dtype = torch.float32):
        super().__init__()
        self.linear = ColumnParallelLinear(in_features=in_features, out_features=out_features, parallel_output=parallel_output,
                                           topology=topology, dtype=dtype, bias=True)
        self.act_fn = act_fn

    def forward(self, x: Union[MLPLayerIO, MNISTDatasetBatch]) -> MLPLayerIO:
        return MLPLayerIO(activations=self.act_fn(self.linear(_inputs(x))))


class MLPLinearRowParallel(MLPBaseLayer):
    def __init__(self, in_features: int, out_features: int, topology: Topology, act_fn: Callable = lambda x: x,
                 dtype: torch.dtype = torch.float32):
        super().__init__()
        self.linear = RowParallelLinear(in_features=in_features, out_features=out_features, parallel_input=True,
                                        topology=topology, dtype=dtype, bias=True)
        self.act_fn = act_fn

    def forward(self, x: Union[MLPLayerIO, MNISTDatasetBatch]) -> MLPLayerIO:
        return MLPLayerIO(activations=self.act_fn(self.linear(_inputs(x))))


def loss_function(output: MLPLayerIO, batch: MNISTDatasetBatch) -> tuple[torch.Tensor, dict[str, torch.Tensor]]:
    assert batch.targets is not None
    target = batch.targets.long()
    logits = output.activations.float()
    loss = F.cross_entropy(logits, target)
    accuracy = (logits.argmax(dim=1) == target).float().mean()
    return loss, {"accuracy": accuracy.detach()}


def metrics_aggregation_fn(topology: Topology, metrics: list[dict[str, torch.Tensor]]) -> dict[str, torch.Tensor]:
    out = {}
    for k in metrics[0]:
        t = torch.stack([torch.as_tensor(m[k], device=topology.device).float() for m in metrics]).mean()
        if topology.config.data_parallel_size > 1:
            torch.distributed.all_reduce(t, group=topology.data_parallel_group)
            t = t / topology.config.data_parallel_size
        out[k] = t
    return out


def init_model(context: MLPContext) -> ParallelModule:
    n_layers = context.config.architecture.n_hidden_layers + 2  # + input and output layers
    hidden = context.config.architecture.hidden_dim
    classes = [MLPLinearColumnParallel, MLPLinearRowParallel]
    specs = []
    for i in range(n_layers):
        kw: dict[str, Any] = {"in_features": hidden if i else 28 * 28,
                              "out_features": hidden if i != n_layers - 1 else 10}
        if i == n_layers - 1 and classes[i % 2] is MLPLinearColumnParallel:
            kw["parallel_output"] = False
        if i != n_layers - 1:
            kw["act_fn"] = F.relu
        specs.append(LayerSpec(module_class=classes[i % 2], topology=context.topology, dtype=torch.float16, **kw))
    return ParallelModule(layer_specs=specs, topology=context.topology, profiler_config=context.config.profiler)


def init_optimizer(context: MLPContext, model: ParallelModule) -> BaseOptimizer:
    group = OptimizerParamGroup(
        named_parameters_with_meta=list(model.named_parameters_with_meta()),
        config=OptimizerParamGroupConfig(name="weight_decay_params", weight_decay=context.config.training.weight_decay,
                                         learning_rate_scheduler=context.config.learning_rate_scheduler),
    )
    return Optimizer(config=context.config.optimizer, parameter_groups=[group], topology=context.topology)
