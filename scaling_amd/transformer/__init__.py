"""Transformer suite (reference ``src/scaling/transformer``): config, data, model, training, inference."""
from .context import TransformerConfig, TransformerContext
from .data import TextBlendedDataset, TextDataset, TextDatasetItem
from .model import TransformerLayerIO, TransformerParallelModule, init_model, init_optimizer

__all__ = [
    "TextBlendedDataset",
    "TextDataset",
    "TextDatasetItem",
    "TransformerConfig",
    "TransformerContext",
    "TransformerLayerIO",
    "TransformerParallelModule",
    "init_model",
    "init_optimizer",
]
