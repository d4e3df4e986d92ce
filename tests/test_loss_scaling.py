"""fp16 + dynamic loss scaling as a tested training mode (reference: ``src/scaling/core/optimizer/loss_scaler.py:83-113``,
``tests/core/test_training/test_training.py:160-200``, ``tests/transformer/test_training.py:70-120,182-185``).

* the scaler's state machine (hysteresis, window growth, ``min_scale``, ``consecutive_hysteresis``) against an
  independently written transition table;
* an inf gradient injected on ONE rank under DP2 and TP2 (gloo): every rank skips the step, the scale shrinks on
  every rank, parameters and AdamW state stay untouched, the next clean step updates;
* fp16 end-to-end training with the scaler through the full entry point, checkpoint at step 6, bit-exact resume
  (also with an initial scale large enough that the first steps overflow and are skipped)."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from tests.dist_utils import make_topology, run_distributed
from tests.test_training import _config, _make_data, _run

pytestmark = pytest.mark.cpu


def _expected(overflows, init, factor, window, hyst, consecutive, min_scale):
    """Plain re-statement of the DeepSpeed dynamic-scaler rules (not the implementation under test)."""
    scale, h, clean = init, hyst, 0
    out = []
    for ov in overflows:
        if ov:
            if h <= 1:
                scale = max(scale / factor, min_scale)
            else:
                h -= 1
            clean = 0
        else:
            if consecutive:
                h = hyst
            if clean > 0 and clean % window == 0:
                if not consecutive:
                    h = hyst
                scale *= factor
            clean += 1
        out.append((scale, h, clean))
    return out


@pytest.mark.parametrize("hyst", [1, 2, 3])
@pytest.mark.parametrize("consecutive", [False, True])
@pytest.mark.parametrize("window", [1, 3])
def test_loss_scaler_state_machine(hyst, consecutive, window):
    from scaling_amd.core import LossScaler, LossScalerConfig

    cfg = LossScalerConfig(enable=True, initial_scale=64.0, window=window, hysteresis=hyst,
                           consecutive_hysteresis=consecutive, min_scale=2.0, factor=2.0)
    ls = LossScaler(cfg)
    rng = np.random.RandomState(hyst * 10 + window + int(consecutive))
    pattern = [True, True, False, True, False, False, False, False, True, True, True, True, True, True, True,
               False] + list(rng.rand(40) < 0.35)
    exp = _expected(pattern, 64.0, 2.0, window, hyst, consecutive, 2.0)
    for ov, (scale, h, clean) in zip(pattern, exp):
        out = ls.step(bool(ov))
        assert out.overflow == bool(ov)
        assert out.current_loss_scale == scale
        assert out.no_overflow_steps == clean
        st = ls.state_dict()
        assert st["current_hysteresis"] == h and st["current_scale"] == scale
    assert min(s for s, _, _ in exp) >= 2.0  # min_scale bound reached and held by the long overflow run
    # state round trip
    ls2 = LossScaler(cfg)
    ls2.load_state_dict(ls.state_dict())
    assert ls2.step(False) == ls.step(False)


def test_loss_scaler_disabled_is_inert():
    from scaling_amd.core import LossScaler, LossScalerConfig

    ls = LossScaler(LossScalerConfig(enable=False, initial_scale=1024.0))
    x = torch.tensor(3.0)
    assert ls.scale_loss(x) is x and ls.current_scale == 1.0
    assert ls.step(True) == (None, None, None)


def _inject_case(mp: int, inject_rank: int):
    from scaling_amd.core import (CoreParameterMeta, LearningRateSchedulerConfig, LossScalerConfig, Optimizer,
                                  OptimizerConfig, OptimizerParamGroup, OptimizerParamGroupConfig)

    topo = make_topology(model_parallel_size=mp)
    rank = torch.distributed.get_rank()
    g = torch.Generator().manual_seed(3)
    params = []
    for i, s in enumerate([(6, 5), (17,), (4, 4, 3)]):
        p = torch.nn.Parameter(torch.randn(*s, generator=g))
        CoreParameterMeta.register_on_parameter(p, is_model_parallel=False, layer_index=i, parameter_name=f"w{i}")
        params.append(p)
    group = OptimizerParamGroup(
        [(f"w{i}", p, p.core_parameter_meta) for i, p in enumerate(params)],
        OptimizerParamGroupConfig(name="g", weight_decay=0.1, learning_rate_scheduler=LearningRateSchedulerConfig(
            learning_rate=0.05, learning_rate_decay_style="constant")),
    )
    cfg = OptimizerConfig(beta1=0.9, beta2=0.95, eps=1e-8, gradient_clipping=1.0, zero=True, grad_bucket_numel=32,
                          loss_scaler=LossScalerConfig(enable=True, initial_scale=1024.0, hysteresis=1, window=100))
    opt = Optimizer(cfg, [group], topo)
    before = [p.detach().clone() for p in params]
    # step 1: an inf on one rank only (gradients carry the loss scale, as after a scaled backward)
    for i, p in enumerate(params):
        p.grad.copy_(torch.full_like(p, 0.01 * (i + 1)) * 1024.0)
    if rank == inject_rank:
        params[1].grad[3] = float("inf")
    out = opt.step()
    assert out.overflow is True and out.global_grad_norm is None
    assert opt.loss_scaler.current_scale == 512.0
    for p, b in zip(params, before):
        assert torch.equal(p.detach(), b)
    assert all(float(g.exp_avg.abs().sum()) == 0.0 for g in opt.parameter_groups)  # AdamW state untouched
    # step 2: clean gradients (scaled by the shrunk scale) update every rank identically
    for i, p in enumerate(params):
        p.grad.copy_(torch.full_like(p, 0.01 * (i + 1)) * 512.0)
    out = opt.step()
    assert out.overflow is False and out.global_grad_norm is not None
    want = math.sqrt(sum(((0.01 * (i + 1)) ** 2) * p.numel() for i, p in enumerate(params)))
    assert abs(out.global_grad_norm - want) < 1e-5
    assert any(not torch.equal(p.detach(), b) for p, b in zip(params, before))
    return [p.detach().flatten().tolist() for p in params]


@pytest.mark.parametrize("mp,inject_rank", [(1, 1), (2, 1), (1, 0)])
def test_injected_overflow_skips_step_on_every_rank(mp, inject_rank):
    res = run_distributed(_inject_case, 2, mp=mp, inject_rank=inject_rank)
    for a, b in zip(res[0], res[1]):  # replicas stay identical
        assert a == b


def _fp16_config(tmp, mp, pp, world, initial_scale):
    cfg = _config(tmp, mp, pp, world, precision="float16")
    cfg["optimizer"]["loss_scaler"] = {"enable": True, "initial_scale": initial_scale, "window": 3, "hysteresis": 1}
    return cfg


@pytest.mark.parametrize("mp,pp,world,initial_scale", [(1, 1, 1, 16.0), (1, 1, 2, 16.0), (2, 1, 2, 16.0),
                                                        (1, 2, 2, 16.0), (1, 1, 2, 2.0 ** 40)])
def test_fp16_loss_scaling_train_and_resume_bit_exact(tmp_path, mp, pp, world, initial_scale):
    _make_data(tmp_path / "data")
    cfg = _fp16_config(tmp_path, mp, pp, world, initial_scale)
    full = _run(tmp_path, cfg, world, "full")
    assert len(full) == 10
    assert all(np.isfinite(m["training/loss"]) for m in full)
    scales = [m["training/current_loss_scale"] for m in full]
    if initial_scale > 1e9:  # fp16 gradients of a 2^40-scaled loss overflow: steps are skipped, the scale shrinks
        assert any(m["training/overflow"] for m in full)
        assert scales[-1] < initial_scale
    else:  # a window of 3 clean steps grows the scale
        assert max(scales) > initial_scale
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, cfg, world, "resumed")
    assert [m["training/loss"] for m in resumed] == [m["training/loss"] for m in full[-4:]]
    assert [m["training/current_loss_scale"] for m in resumed] == scales[-4:]
