"""Transformer suite (reference ``src/scaling/transformer``): config, data, model, training, inference."""
from .context import TransformerConfig, TransformerContext
from .data import (
    FinetuningChatBlendedDataset,
    FinetuningChatDataset,
    FinetuningTextBlendedDataset,
    FinetuningTextDataset,
    LegacyBlendedDataset,
    TextBlendedDataset,
    TextDataset,
    TextDatasetItem,
)
from .model import TransformerLayerIO, TransformerParallelModule, init_model, init_optimizer

__all__ = [
    "FinetuningChatBlendedDataset",
    "FinetuningChatDataset",
    "FinetuningTextBlendedDataset",
    "FinetuningTextDataset",
    "LegacyBlendedDataset",
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
