"""Optimizer: fused AdamW over flat bucketed buffers vs torch.optim.AdamW; ZeRO-1 over 2 data-parallel
ranks vs the single-rank update on the averaged gradient; checkpoint round trip.  (Reference:
tests/core/test_optimizer/test_adamw.py.)"""
import pytest
import torch

from tests.dist_utils import make_topology, run_distributed

pytestmark = pytest.mark.cpu

SHAPES = [(5, 7), (11,), (3, 4, 6), (129,)]


def _make_params(seed=0):
    from scaling_amd.core import CoreParameterMeta

    g = torch.Generator().manual_seed(seed)
    params = []
    for i, s in enumerate(SHAPES):
        p = torch.nn.Parameter(torch.randn(*s, generator=g))
        CoreParameterMeta.register_on_parameter(p, is_model_parallel=False, layer_index=i, parameter_name=f"w{i}")
        params.append(p)
    return params


def _grads(step, rank, seed=1):
    g = torch.Generator().manual_seed(seed + 1000 * step + 17 * rank)
    return [torch.randn(*s, generator=g) for s in SHAPES]


def _opt(params, topo, zero, clip, bucket, lr=0.05, wd=0.1):
    from scaling_amd.core import (LearningRateSchedulerConfig, Optimizer, OptimizerConfig, OptimizerParamGroup,
                                  OptimizerParamGroupConfig)

    group = OptimizerParamGroup(
        [(f"w{i}", p, p.core_parameter_meta) for i, p in enumerate(params)],
        OptimizerParamGroupConfig(name="g", weight_decay=wd,
                                  learning_rate_scheduler=LearningRateSchedulerConfig(learning_rate=lr, learning_rate_decay_style="constant")),
    )
    cfg = OptimizerConfig(beta1=0.9, beta2=0.95, eps=1e-8, gradient_clipping=clip, zero=zero, grad_bucket_numel=bucket)
    return Optimizer(cfg, [group], topo)


def _adamw_case(zero, clip, bucket, steps=3):
    topo = make_topology()
    dp = topo.config.data_parallel_size
    params = _make_params()
    ref = [torch.nn.Parameter(p.detach().clone()) for p in params]
    opt = _opt(params, topo, zero, clip, bucket)
    ref_opt = torch.optim.AdamW(ref, lr=0.05, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(steps):
        mine = _grads(step, topo.data_parallel_rank)
        for p, g in zip(params, mine):
            p.grad.copy_(g)  # grads are views into the flat buffer
        avg = [sum(gs) / dp for gs in zip(*[_grads(step, r) for r in range(dp)])]
        out = opt.step()
        norm = torch.sqrt(sum((g.double() ** 2).sum() for g in avg)).item()
        assert abs(out.global_grad_norm - norm) < 1e-5 * max(1.0, norm)
        scale = min(1.0, clip / norm) if clip > 0 else 1.0
        for r, g in zip(ref, avg):
            r.grad = g * scale
        ref_opt.step()
        for p, r in zip(params, ref):
            torch.testing.assert_close(p.detach(), r.detach(), rtol=1e-5, atol=1e-6)
    return True


@pytest.mark.parametrize("clip", [0.0, 1.0])
@pytest.mark.parametrize("bucket", [64, 1 << 20])
def test_adamw_matches_torch(clip, bucket):
    assert all(run_distributed(_adamw_case, 1, zero=False, clip=clip, bucket=bucket).values())


@pytest.mark.parametrize("bucket", [64, 1 << 20])
def test_zero1_dp2_matches_single_rank_update(bucket):
    assert all(run_distributed(_adamw_case, 2, zero=True, clip=1.0, bucket=bucket).values())


def test_dp2_without_zero():
    assert all(run_distributed(_adamw_case, 2, zero=False, clip=1.0, bucket=256).values())


def _ckpt_case(tmp):
    from pathlib import Path

    topo = make_topology()
    params = _make_params()
    opt = _opt(params, topo, True, 1.0, 64)
    for step in range(2):
        for p, g in zip(params, _grads(step, topo.data_parallel_rank)):
            p.grad.copy_(g)
        opt.step()
    opt.save_checkpoint(Path(tmp))
    torch.distributed.barrier()  # files are written by data-parallel rank 0
    snap = [p.detach().clone() for p in params]
    # fresh optimizer on perturbed params, load, one more identical step on both
    params2 = _make_params(seed=5)
    with torch.no_grad():
        for p, s in zip(params2, snap):
            p.copy_(s)
    opt2 = _opt(params2, topo, True, 1.0, 64)
    opt2.load_checkpoint(Path(tmp))
    for o, ps in ((opt, params), (opt2, params2)):
        for p, g in zip(ps, _grads(7, topo.data_parallel_rank)):
            p.grad.copy_(g)
        o.step()
    for a, b in zip(params, params2):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=0, atol=0)
    return True


def test_optimizer_checkpoint_roundtrip_zero_dp2(tmp_path):
    assert all(run_distributed(_ckpt_case, 2, tmp=str(tmp_path)).values())
