"""Final norm as its own pipeline layer (reference ``model/layers/layernorm.py``)."""
from __future__ import annotations

from typing import Optional

from ....core import Topology, get_norm
from ...context.config import TransformerArchitectureConfig
from .base import TransformerLayerBaseIO, TransformerLayerIO
from .embedding import _device


class LayerNormWrapper(TransformerLayerBaseIO):
    def __init__(self, architecture_config: TransformerArchitectureConfig, layer_index: int, topology: Optional[Topology] = None):
        super().__init__()
        cfg = architecture_config
        self.topology = topology
        self.architecture_config = cfg
        self.norm = get_norm(cfg.norm_type, cfg.layernorm, cfg.hidden_size, _device(topology), cfg.precision.dtype,
                             getattr(cfg.bitfit_bias_config, "name", None), topology)
        self.layer_index = layer_index

    def forward(self, x: TransformerLayerIO) -> TransformerLayerIO:
        if x.residual_branch is not None and hasattr(self.norm, "forward_add"):  # last layer's pending MLP residual add
            act = self.norm.forward_add(x.activations, x.residual_branch)[1]
        else:
            act = self.norm(x.hidden())
        st = x.inference_settings
        if st is not None and (self.layer_index + 1) in st.embedding_layers:
            assert x.embeddings is not None
            x.embeddings[st.embedding_layers.index(self.layer_index + 1)] = act
        return x.derive(act, attention_scores_manipulation=None)
