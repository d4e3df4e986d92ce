"""Vocab-parallel embedding (reference ``vocab_parallel_embedding.py:19-147``).

On GPU the masked lookup + zeroing runs in one HIP kernel (``scaling_amd.ops.embedding``) and the
backward is a deterministic sorted segment-sum, so no float atomics touch the table.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ....ops import embedding as emb_ops
from ...topology import Topology
from ..parameter_meta import CoreParameterMeta
from .utils import all_reduce, all_reduce_scatter_to_sequence_parallel, get_device


class VocabParallelEmbedding(torch.nn.Module):
    def __init__(
        self,
        num_embeddings: int,
        embedding_dim: int,
        finetunable_token_ids: list[int],
        device: Optional[torch.device] = None,
        dtype: torch.dtype = torch.float32,
        topology: Optional[Topology] = None,
        init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_,
    ) -> None:
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self._device = get_device(topology=topology, device=device)
        self.dtype = dtype
        self.topology = topology
        self.init_method = init_method
        self.model_parallel_size = 1 if topology is None else topology.config.model_parallel_size
        assert num_embeddings % self.model_parallel_size == 0, (
            f"cannot parallelize embedding, num_embeddings ({num_embeddings}) "
            f"needs to be divisible by model parallel size ({self.model_parallel_size})"
        )
        self.vocab_size_per_partition = num_embeddings // self.model_parallel_size
        rank = 0 if topology is None else topology.model_parallel_rank
        self.vocab_start_index = rank * self.vocab_size_per_partition
        self.vocab_end_index = self.vocab_start_index + self.vocab_size_per_partition
        self.weight = torch.nn.Parameter(
            torch.empty(self.vocab_size_per_partition, embedding_dim, device=self._device, dtype=dtype)
        )
        init_method(self.weight)
        CoreParameterMeta.register_on_parameter(self.weight, is_model_parallel=True, model_parallel_dimension=0)
        if len(finetunable_token_ids) > 0:
            mask = torch.zeros(self.vocab_size_per_partition, 1, device=self._device, dtype=dtype)
            for token_id in finetunable_token_ids:
                if self.vocab_start_index <= token_id < self.vocab_end_index:
                    mask[token_id - self.vocab_start_index] = 1
            self.register_buffer("_finetune_mask", mask, persistent=False)
            self.weight.register_hook(lambda g: None if g is None else g * self._finetune_mask)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = emb_ops.vocab_embedding(x, self.weight, self.vocab_start_index, self.vocab_end_index)
        if self.model_parallel_size > 1:
            assert self.topology is not None
            if self.topology.config.sequence_parallel:
                return all_reduce_scatter_to_sequence_parallel(out, topology=self.topology)
            return all_reduce(out, topology=self.topology)
        return out
