"""One GEMM for several ColumnParallelLinear modules that read the same input.

The reference issues a separate GEMM and a separate TP backward all-reduce per module (separate
q/k/v for GQA, ``dense_in``/``siglu_weight`` for SwiGLU: ``column_parallel_linear.py:137-139``).
``fused_column_linear`` keeps the modules (and therefore parameter names / checkpoint keys) but runs
``x @ [W_1; W_2; ...]^T`` as one hipBLASLt GEMM, computes all weight gradients with one GEMM
(accumulated in place into the flat gradient buffer, see ``main_grad.py``), and issues a single
all-reduce for the input gradient.
"""
from __future__ import annotations

from typing import Any, Sequence

import torch

from .main_grad import multi_linear
from .utils import tp_input_grad_group


def fused_column_linear(x: torch.Tensor, modules: Sequence[torch.nn.Module], topology: Any) -> torch.Tensor:
    """Apply several ColumnParallelLinear (parallel_output=True) modules to the same input with one GEMM."""
    weights = [m.weight for m in modules]  # type: ignore[attr-defined]
    biases = [getattr(m, "bias_param", None) for m in modules]
    if any(b is None for b in biases):
        biases = [None] * len(modules)
    return multi_linear(x, weights, biases, tp_group=tp_input_grad_group(topology))
