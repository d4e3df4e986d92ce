"""LM head tied to the input embedding (reference ``model/layers/lm_head_tied.py``).

The head owns a ``VocabParallelEmbedding`` whose weight the ``TiedLayerIndex`` of the parallel module ties to
the input embedding; its logits are ``x @ E^T`` through the framework GEMM (hipBLASLt forward / dgrad, HIP wgrad
into the main-grad buffer).  Under tensor parallelism the logits stay vocab-sharded while training (the fused
vocab-parallel cross-entropy consumes them) and are all-gathered in eval, as in ``lm_head.TransformerLMHead``.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ....core import Topology, VocabParallelEmbedding
from ....core.nn.linear.utils import copy_to_tensor_model_parallel_region
from ....ops.gemm import linear as gemm_linear
from ...context.config import TransformerArchitectureConfig
from .base import TransformerLayerBaseIO, TransformerLayerIO
from .embedding import _device


class TransformerLMHeadTied(TransformerLayerBaseIO):
    def __init__(self, architecture_config: TransformerArchitectureConfig,
                 init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
                 topology: Optional[Topology] = None):
        super().__init__()
        cfg = architecture_config
        self.topology = topology
        self.embedding = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, topology=topology,
                                                device=None if topology is not None else _device(topology),
                                                dtype=cfg.precision.dtype, init_method=init_method,
                                                finetunable_token_ids=cfg.finetunable_token_ids)
        tp = 1 if topology is None else topology.config.model_parallel_size
        self.vocab_per_rank = cfg.vocab_size // tp

    def forward(self, x: TransformerLayerIO) -> TransformerLayerIO:
        from .lm_head import _finish

        act = x.activations
        if self.topology is not None and self.topology.config.model_parallel_size > 1:
            act = copy_to_tensor_model_parallel_region(act, topology=self.topology)
        return _finish(self, x, gemm_linear(act, self.embedding.weight), self.vocab_per_rank)


__all__ = ["TransformerLMHeadTied"]
