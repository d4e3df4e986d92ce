from .attention import (
    KVCache,
    ParallelSelfAttention,
    RelativePositionEmbeddingType,
    cumulative_seq_lengths_to_dense_attention_mask,
    get_max_seq_length,
    multi_head_attention,
    repeat_kv,
    split_tensor_along_last_dim,
)

__all__ = [
    "KVCache",
    "ParallelSelfAttention",
    "RelativePositionEmbeddingType",
    "cumulative_seq_lengths_to_dense_attention_mask",
    "get_max_seq_length",
    "multi_head_attention",
    "repeat_kv",
    "split_tensor_along_last_dim",
]
