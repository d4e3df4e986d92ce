"""Reference-compatible names for the TP/SP region functions (implemented in ``scaling_amd.parallel.tp``).

Reference: ``src/scaling/core/nn/linear/utils.py:195-383``.
"""
from ....parallel.tp import (  # noqa: F401
    all_concat,
    all_reduce,
    all_reduce_scatter_to_sequence_parallel,
    all_shard,
    copy_to_tensor_model_parallel_region,
    gather_from_sequence_parallel_region,
    get_device,
    raw_all_gather_cat,
    raw_all_reduce,
    raw_gather_seq,
    raw_reduce_scatter_seq,
    raw_shard,
    tp_input_grad_group,
)
