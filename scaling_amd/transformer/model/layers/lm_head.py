"""LM heads (reference ``model/layers/lm_head.py`` and ``lm_head_tied.py``).

Training with tensor parallelism keeps the logits vocab-sharded (``parallel_output``) and tags the
layer IO so the loss runs the fused vocab-parallel cross-entropy — the ``[b*s, V]`` all-gather of the
reference is skipped.  In eval/inference mode the logits are all-gathered as in the reference.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ....core import ColumnParallelLinear, Topology
from ....core.nn.linear.utils import all_concat
from ...context.config import TransformerArchitectureConfig
from .base import TransformerLayerBaseIO, TransformerLayerIO
from .embedding import _device


def _finish(self: torch.nn.Module, x: TransformerLayerIO, logits: torch.Tensor, vocab_per_rank: int) -> TransformerLayerIO:
    topo = self.topology
    tp = 1 if topo is None else topo.config.model_parallel_size
    if tp > 1 and not self.training:
        logits = all_concat(logits, dim=-1, topology=topo)
    out = x.derive(logits, attention_scores_manipulation=None)
    if tp > 1 and self.training:
        out.vocab_parallel = (topo.model_parallel_rank * vocab_per_rank, topo.model_parallel_group, tp)
    return out


class TransformerLMHead(TransformerLayerBaseIO):
    def __init__(self, architecture_config: TransformerArchitectureConfig,
                 init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
                 topology: Optional[Topology] = None):
        super().__init__()
        cfg = architecture_config
        self.topology = topology
        self.linear = ColumnParallelLinear(cfg.hidden_size, cfg.vocab_size, bias=False, topology=topology,
                                           device=None if topology is not None else _device(topology),
                                           dtype=cfg.precision.dtype, init_method=init_method, parallel_output=True)
        tp = 1 if topology is None else topology.config.model_parallel_size
        self.vocab_per_rank = cfg.vocab_size // tp
        if cfg.finetunable_token_ids:
            rank = 0 if topology is None else topology.model_parallel_rank
            mask = torch.zeros(self.vocab_per_rank, 1, dtype=self.linear.weight.dtype, device=self.linear.weight.device)
            for t in cfg.finetunable_token_ids:
                if rank * self.vocab_per_rank <= t < (rank + 1) * self.vocab_per_rank:
                    mask[t - rank * self.vocab_per_rank] = 1
            self.register_buffer("_finetune_mask", mask, persistent=False)
            # honoured by the GEMM-fused weight-gradient path (core/nn/linear/main_grad.py)
            self.linear.weight._sa_grad_row_mask = self._finetune_mask  # type: ignore[attr-defined]

    def forward(self, x: TransformerLayerIO) -> TransformerLayerIO:
        return _finish(self, x, self.linear(x.activations), self.vocab_per_rank)


from .lm_head_tied import TransformerLMHeadTied  # noqa: E402,F401  (re-export)
