from .layers import *  # noqa: F401,F403
from .model import (
    TransformerParallelModule,
    get_parameter_groups,
    get_transformer_layer_specs,
    init_model,
    init_optimizer,
    loss_function,
    metrics_aggregation_fn,
)

__all__ = [
    "TransformerParallelModule",
    "get_parameter_groups",
    "get_transformer_layer_specs",
    "init_model",
    "init_optimizer",
    "loss_function",
    "metrics_aggregation_fn",
]
