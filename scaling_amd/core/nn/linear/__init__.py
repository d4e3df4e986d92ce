from .column_parallel_linear import ColumnParallelLinear
from .row_parallel_linear import RowParallelLinear
from .utils import (
    all_concat,
    all_reduce,
    all_reduce_scatter_to_sequence_parallel,
    all_shard,
    copy_to_tensor_model_parallel_region,
    gather_from_sequence_parallel_region,
    get_device,
)
from .vocab_parallel_embedding import VocabParallelEmbedding

__all__ = [
    "ColumnParallelLinear",
    "RowParallelLinear",
    "VocabParallelEmbedding",
    "all_concat",
    "all_reduce",
    "all_reduce_scatter_to_sequence_parallel",
    "all_shard",
    "copy_to_tensor_model_parallel_region",
    "gather_from_sequence_parallel_region",
    "get_device",
]
