"""TP input-gradient all-reduce overlapped with the weight-gradient GEMM (gloo, 2 ranks): the all-reduce of
dX is issued asynchronously before the wgrad GEMM and waited for after it, and the gradients equal the
unfused ``copy_to`` region + linear composition."""
from __future__ import annotations

import pytest
import torch

from tests.dist_utils import make_topology, run_distributed

pytestmark = pytest.mark.cpu


def _case():
    import torch.distributed as dist

    from scaling_amd.core.nn.linear import ColumnParallelLinear, main_grad
    from scaling_amd.core.nn.linear.fused import fused_column_linear
    from scaling_amd.core.nn.linear.utils import copy_to_tensor_model_parallel_region

    topo = make_topology(model_parallel_size=2)
    torch.manual_seed(0)  # same input on both ranks, as in a TP group
    x = torch.randn(3, 8, 32)
    mods = [ColumnParallelLinear(32, 16, bias=True, topology=topo, parallel_output=True) for _ in range(2)]
    for i, m in enumerate(mods):  # rank-specific shards
        torch.manual_seed(100 + 10 * i + topo.model_parallel_rank)
        with torch.no_grad():
            m.weight.normal_()
            m.bias_param.normal_()
    g = torch.randn(3, 8, 8)  # out_features 16 over TP 2

    # reference: copy_to region (all-reduce after the whole backward) + plain linears
    xr = x.clone().requires_grad_(True)
    xc = copy_to_tensor_model_parallel_region(xr, topo)
    ys = [torch.nn.functional.linear(xc, m.weight, m.bias_param) for m in mods]
    torch.autograd.backward(ys, [g, 2 * g])
    ref_dx = xr.grad.clone()
    ref_dw = [m.weight.grad.clone() for m in mods]
    for m in mods:
        m.weight.grad = None
        m.bias_param.grad = None

    events = []
    real_ar, real_wgrad = dist.all_reduce, main_grad.wgrad

    class _Work:
        def __init__(self, w):
            self.w = w

        def wait(self):
            events.append("wait")
            return self.w.wait()

    def ar(t, *a, async_op=False, **k):
        events.append("all_reduce_async" if async_op else "all_reduce")
        w = real_ar(t, *a, async_op=async_op, **k)
        return _Work(w) if async_op else w

    def wg(*a, **k):
        events.append("wgrad")
        return real_wgrad(*a, **k)

    dist.all_reduce, main_grad.wgrad = ar, wg
    try:
        # single column-parallel module
        x1 = x.clone().requires_grad_(True)
        mods[0](x1).backward(g)
        single = list(events)
        events.clear()
        for m in mods:
            m.weight.grad = None
            m.bias_param.grad = None
        # two modules fused into one GEMM (q/k/v, SwiGLU style): one all-reduce for both
        x2 = x.clone().requires_grad_(True)
        y = fused_column_linear(x2, mods, topo)
        y.backward(torch.cat([g, 2 * g], dim=-1))
        fused = list(events)
    finally:
        dist.all_reduce, main_grad.wgrad = real_ar, real_wgrad
    assert single == ["all_reduce_async", "wgrad", "wait"], single
    assert fused == ["all_reduce_async", "wgrad", "wait"], fused
    torch.testing.assert_close(x2.grad, ref_dx, rtol=1e-5, atol=1e-5)
    for m, r in zip(mods, ref_dw):
        torch.testing.assert_close(m.weight.grad, r, rtol=1e-5, atol=1e-5)
    return True


def test_tp_input_grad_allreduce_overlaps_wgrad():
    assert all(run_distributed(_case, 2).values())


def _row_chunked_case(sp: bool, chunks: int):
    """RowParallelLinear with ``tensor_parallel_comm_chunks``: the piecewise GEMM + all-reduce (or SP
    reduce-scatter into the reference's flat token partition) equals the one-GEMM-then-collective path, forward
    and backward (input gradient and weight gradient)."""
    from scaling_amd.core.nn.linear import RowParallelLinear

    topo = make_topology(model_parallel_size=2, sequence_parallel=sp)
    rank = topo.model_parallel_rank
    m = RowParallelLinear(32, 24, bias=False, topology=topo, parallel_input=True, parallel_output=sp)
    torch.manual_seed(7 + rank)
    with torch.no_grad():
        m.weight.normal_()
    x = torch.randn(4, 16, 16, requires_grad=True)  # [b, s, in/tp]: this rank's input shard
    outs = {}
    for c in (1, chunks):
        object.__setattr__(topo.config, "tensor_parallel_comm_chunks", c)  # frozen config: test-only override
        x.grad = None
        m.weight.grad = None
        y = m.forward_sequence_parallel(x) if sp else m(x)
        torch.manual_seed(99 + rank)
        g = torch.randn_like(y)
        (y * g).sum().backward()
        outs[c] = (y.detach().clone(), x.grad.clone(), m.weight.grad.clone())
    for a, b in zip(outs[1], outs[chunks]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    assert outs[1][0].shape == ((4, 8, 24) if sp else (4, 16, 24))
    return True


@pytest.mark.parametrize("sp,chunks", [(False, 2), (False, 4), (True, 2), (True, 4)])
def test_row_parallel_chunked_matches_unchunked(sp, chunks):
    assert all(run_distributed(_row_chunked_case, 2, sp=sp, chunks=chunks).values())


def _chunked_save_matmuls_case(sp: bool):
    """``tensor_parallel_comm_chunks`` > 1 under ``every_layer_save_matmuls``: the checkpoint recompute replays the
    piecewise GEMM + collective output instead of running it again (one forward call, no second collective), and the
    gradients equal plain per-layer checkpointing."""
    import scaling_amd.core.nn.linear.tp_overlap as tpo
    from scaling_amd.core.nn.linear import RowParallelLinear
    from scaling_amd.core.nn.parallel_module.activation_checkpointing import checkpoint_with_rng

    topo = make_topology(model_parallel_size=2, sequence_parallel=sp, tensor_parallel_comm_chunks=2)
    rank = topo.model_parallel_rank
    m = RowParallelLinear(32, 24, bias=False, topology=topo, parallel_input=True, parallel_output=sp)
    torch.manual_seed(7 + rank)
    with torch.no_grad():
        m.weight.normal_()
    real = tpo._chunked_forward
    calls = []

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)

    grads = {}
    for keep in (False, True):
        calls.clear()
        m.weight.grad = None
        torch.manual_seed(11 + rank)
        x = torch.randn(4, 16, 16, requires_grad=True)
        fn = (lambda t: m.forward_sequence_parallel(t)) if sp else (lambda t: m(t))
        tpo._chunked_forward = counting
        try:
            y = checkpoint_with_rng(fn, topo, True, x, keep_gemms=keep)
            (y * y).sum().backward()
        finally:
            tpo._chunked_forward = real
        assert len(calls) == (1 if keep else 2), (keep, len(calls))
        grads[keep] = (x.grad.clone(), m.weight.grad.clone())
    for a, b in zip(grads[False], grads[True]):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    return True


@pytest.mark.parametrize("sp", [False, True])
def test_row_parallel_chunked_under_save_matmuls(sp):
    assert all(run_distributed(_chunked_save_matmuls_case, 2, sp=sp).values())
