"""Image encoder = CLIP RN50x16 tower → linear projection to the hidden size → dropout → optional
LayerNorm (reference ``model/image_encoder/image_encoder.py``).  144 tokens per 384x384 image."""
from __future__ import annotations

from typing import Optional

import torch

from ....core import LayerNorm, LayerNormConfig
from .clip import ClipModifiedResNet

IMAGE_SIZE = (384, 384)
DOWNSAMPLE = 32


class ImageEncoder(torch.nn.Module):
    def __init__(self, out_features: int, device: torch.device, dropout_p: float = 0.0,
                 layernorm_config: Optional[LayerNormConfig] = None, image_encoder: str = "ClipRN50x16",
                 dtype: torch.dtype = torch.float32):
        super().__init__()
        assert image_encoder == "ClipRN50x16", "only clip implemented"
        self.input_encoder = ClipModifiedResNet(layers=[6, 8, 18, 8], num_init_channels=96).to(dtype).to(device)
        self.image_encoder_image_size = IMAGE_SIZE
        self.num_tokens = (IMAGE_SIZE[0] // DOWNSAMPLE) * (IMAGE_SIZE[1] // DOWNSAMPLE)
        self.input_encoder_output_dim = 3072
        self.do_token_reshape = False
        self.reshape_shape = (self.num_tokens, self.input_encoder_output_dim)
        self.proj = torch.nn.Linear(self.input_encoder_output_dim, out_features, device=device, dtype=dtype)
        self.dropout = torch.nn.Dropout(dropout_p)
        self.has_layernorm = layernorm_config is not None
        if layernorm_config is not None:
            self.layernorm = LayerNorm(config=layernorm_config, normalized_shape=out_features, device=device, dtype=dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.dropout(self.proj(self.input_encoder(x)))
        return self.layernorm(x) if self.has_layernorm else x
