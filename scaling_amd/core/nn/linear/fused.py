"""One GEMM for several ColumnParallelLinear modules that read the same input.

The reference issues a separate GEMM and a separate TP backward all-reduce per module (separate
q/k/v for GQA, ``dense_in``/``siglu_weight`` for SwiGLU: ``column_parallel_linear.py:137-139``).
``fused_column_linear`` keeps the modules (and therefore parameter names / checkpoint keys) but runs
``x @ [W_1; W_2; ...]^T`` as one hipBLASLt GEMM, computes all weight gradients with one GEMM, and
issues a single all-reduce for the input gradient.
"""
from __future__ import annotations

from typing import Any, Optional, Sequence

import torch

from .utils import copy_to_tensor_model_parallel_region


class _FusedColumnLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x: torch.Tensor, *params: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        n = len(params) // 2
        weights, biases = params[:n], params[n:]
        w = torch.cat(weights, dim=0) if n > 1 else weights[0]
        has_bias = biases[0] is not None
        b = (torch.cat(biases, dim=0) if n > 1 else biases[0]) if has_bias else None
        out = torch.nn.functional.linear(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.splits = [t.shape[0] for t in weights]
        ctx.has_bias = has_bias
        ctx.n = n
        return out

    @staticmethod
    def backward(ctx: Any, g: torch.Tensor):  # type: ignore[override]
        x, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.matmul(g, w)
        dws: list[Optional[torch.Tensor]] = [None] * ctx.n
        if any(ctx.needs_input_grad[1 : 1 + ctx.n]):
            dw = torch.matmul(g2.t(), x.reshape(-1, x.shape[-1]))
            dws = list(torch.split(dw, ctx.splits, dim=0))
        dbs: list[Optional[torch.Tensor]] = [None] * ctx.n
        if ctx.has_bias and any(ctx.needs_input_grad[1 + ctx.n :]):
            dbs = list(torch.split(g2.sum(0), ctx.splits, dim=0))
        return (dx, *dws, *dbs)


def fused_column_linear(x: torch.Tensor, modules: Sequence[torch.nn.Module], topology: Any) -> torch.Tensor:
    """Apply several ColumnParallelLinear (parallel_output=True) modules to the same input with one GEMM."""
    tp = 1 if topology is None else topology.config.model_parallel_size
    if tp > 1 and not topology.config.sequence_parallel:
        x = copy_to_tensor_model_parallel_region(x, topology=topology)
    weights = [m.weight for m in modules]  # type: ignore[attr-defined]
    biases = [getattr(m, "bias_param", None) for m in modules]
    if any(b is None for b in biases):
        biases = [None] * len(modules)
    return _FusedColumnLinear.apply(x, *weights, *biases)
