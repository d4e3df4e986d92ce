"""Tensor-parallel layers on gloo (world 2) against the same math on merged weights.

Mirrors the reference's tests/core/test_nn/test_parallel_linear.py, test_parallel_embedding.py and the
vocab-parallel loss: shards are gathered from all ranks, the unsharded computation is run locally and
outputs / input gradients / weight gradients are compared.
"""
import pytest
import torch

from tests.dist_utils import make_topology, run_distributed

pytestmark = pytest.mark.cpu


def _gather(t, topo, dim):
    import torch.distributed as dist

    parts = [torch.empty_like(t) for _ in range(topo.config.model_parallel_size)]
    dist.all_gather(parts, t.contiguous(), group=topo.model_parallel_group)
    return torch.cat(parts, dim=dim)


def _linear_case(kind: str, bias: bool, sequence_parallel: bool = False):
    from scaling_amd.core import ColumnParallelLinear, RowParallelLinear

    topo = make_topology(model_parallel_size=2, sequence_parallel=sequence_parallel)
    torch.manual_seed(1234)  # same input on both ranks
    x = torch.randn(3, 8, 16)
    g = torch.randn(3, 8, 24)
    torch.manual_seed(100 + topo.model_parallel_rank)
    if kind == "column":
        layer = ColumnParallelLinear(16, 24, bias=bias, topology=topo, parallel_output=False)
        w_full = _gather(layer.weight.detach(), topo, 0)
        b_full = _gather(layer.bias_param.detach(), topo, 0) if bias else None
    else:
        layer = RowParallelLinear(16, 24, bias=bias, topology=topo, parallel_input=False, parallel_output=False)
        w_full = _gather(layer.weight.detach(), topo, 1)
        b_full = layer.bias_param.detach() if bias else None
    xr = x.clone().requires_grad_(True)
    out = layer(xr)
    out.backward(g)
    xf = x.clone().requires_grad_(True)
    wf = w_full.clone().requires_grad_(True)
    ref = torch.nn.functional.linear(xf, wf, b_full)
    ref.backward(g)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(xr.grad, xf.grad, rtol=1e-5, atol=1e-5)
    dim = 0 if kind == "column" else 1
    torch.testing.assert_close(_gather(layer.weight.grad, topo, dim), wf.grad, rtol=1e-5, atol=1e-5)
    return True


@pytest.mark.parametrize("kind", ["column", "row"])
@pytest.mark.parametrize("bias", [True, False])
def test_parallel_linear_tp2(kind, bias):
    assert all(run_distributed(_linear_case, 2, kind=kind, bias=bias).values())


def _embedding_case():
    from scaling_amd.core import VocabParallelEmbedding

    topo = make_topology(model_parallel_size=2)
    torch.manual_seed(7 + topo.model_parallel_rank)
    emb = VocabParallelEmbedding(64, 16, finetunable_token_ids=[], topology=topo)
    w_full = _gather(emb.weight.detach(), topo, 0)
    torch.manual_seed(0)
    ids = torch.randint(0, 64, (2, 10))
    g = torch.randn(2, 10, 16)
    out = emb(ids)
    out.backward(g)
    wf = w_full.clone().requires_grad_(True)
    ref = torch.nn.functional.embedding(ids, wf)
    ref.backward(g)
    torch.testing.assert_close(out, ref)
    torch.testing.assert_close(_gather(emb.weight.grad, topo, 0), wf.grad)
    return True


def test_vocab_parallel_embedding_tp2():
    assert all(run_distributed(_embedding_case, 2).values())


def _xent_case():
    from scaling_amd.ops.xent import cross_entropy_reference, vocab_parallel_cross_entropy

    topo = make_topology(model_parallel_size=2)
    torch.manual_seed(0)
    logits = torch.randn(12, 40)
    target = torch.randint(0, 40, (12,))
    r = topo.model_parallel_rank
    shard = logits[:, 20 * r : 20 * (r + 1)].clone().requires_grad_(True)
    loss, amax = vocab_parallel_cross_entropy(shard, target, v0=20 * r, group=topo.model_parallel_group, tp=2)
    loss.sum().backward()
    full = logits.clone().requires_grad_(True)
    ref, ref_amax = cross_entropy_reference(full, target)
    ref.sum().backward()
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(amax, ref_amax)
    torch.testing.assert_close(shard.grad, full.grad[:, 20 * r : 20 * (r + 1)], rtol=1e-5, atol=1e-6)
    return True


def test_vocab_parallel_cross_entropy_tp2():
    assert all(run_distributed(_xent_case, 2).values())
