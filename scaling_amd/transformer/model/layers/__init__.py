from .base import TransformerLayerBaseIO, TransformerLayerIO
from .embedding import BaseEmbeddingInput, EmbeddingInput
from .embedding_head import TransformerEmbeddingHead
from .layer import TransformerLayer
from .layernorm import LayerNormWrapper
from .lm_head import TransformerLMHead, TransformerLMHeadTied

__all__ = [
    "BaseEmbeddingInput",
    "EmbeddingInput",
    "LayerNormWrapper",
    "TransformerEmbeddingHead",
    "TransformerLMHead",
    "TransformerLMHeadTied",
    "TransformerLayer",
    "TransformerLayerBaseIO",
    "TransformerLayerIO",
]
