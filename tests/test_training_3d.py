"""3D-parallel end-to-end training on CPU/gloo at world sizes 4 and 8 (reference:
tests/transformer/test_training.py:58-302 and tests/core/test_training/test_training.py:150-235, which
train and resume at (mp, pp, world) = (1, 2, 4) and (2, 2, 4)).

Model: the Llama-style configuration of the benchmark (GQA, SwiGLU, complex RoPE, RMSNorm, untied head)
with ZeRO-1 on, shrunk to CPU size.  Covered:
* bit-exact resume of steps 7-10 for (2,2,4), (1,2,4), (2,1,4) and (2,2,8) — TP, PP and DP all > 1 in
  the last one, which is the BASELINE TP2 x PP2 x DP2 layout;
* layout-change resume into and out of (2,2,8);
* numerics: from one fp32 checkpoint, every resumed step's loss under a TP / PP / DP layout matches the
  single-rank run within 1e-5 (no dropout) — tensor-parallel math and complete data-parallel gradients.
"""
from __future__ import annotations

import copy
from pathlib import Path

import numpy as np
import pytest

from tests.test_training import _config, _make_data, _run

pytestmark = pytest.mark.cpu


def _llama_cfg(tmp: Path, mp: int, pp: int, world: int, acc: int = 2, dropout: bool = True) -> dict:
    cfg = _config(tmp, mp, pp, world, relative_position_embedding_type="rotary_complex", num_layers=4)
    cfg["topology"]["gradient_accumulation_steps"] = acc
    if not dropout:
        a = cfg["transformer_architecture"]
        for k in ("dropout_embedding", "dropout_attention_probs", "dropout_after_attention", "dropout_after_mlp"):
            a[k] = 0.0
    return cfg


def _losses(ms: list) -> list:
    return [m["training/loss"] for m in ms]


@pytest.mark.parametrize("mp,pp,world", [(2, 2, 4), (1, 2, 4), (2, 1, 4), (2, 2, 8)])
def test_3d_train_and_resume_bit_exact(tmp_path, mp, pp, world):
    _make_data(tmp_path / "data")
    cfg = _llama_cfg(tmp_path, mp, pp, world)
    full = _run(tmp_path, cfg, world, "full")
    assert len(full) == 10 and all(np.isfinite(_losses(full)))
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, cfg, world, "resumed")
    assert _losses(resumed) == _losses(full)[-4:]


# (mp, pp, world, acc): the global batch (micro 2 x acc x dp) stays 8 across each change
@pytest.mark.parametrize("before,after", [((1, 1, 2, 2), (2, 2, 8, 2)), ((2, 2, 8, 2), (1, 2, 4, 2)),
                                          ((2, 2, 8, 2), (1, 1, 1, 4))])
def test_3d_layout_change_resume(tmp_path, before, after):
    _make_data(tmp_path / "data")
    full = _run(tmp_path, _llama_cfg(tmp_path, *before[:3], acc=before[3]), before[2], "full")
    c2 = _llama_cfg(tmp_path, *after[:3], acc=after[3])
    c2["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, c2, after[2], "resumed")
    for a, b in zip(_losses(full)[-4:], _losses(resumed)):
        assert abs(a - b) / a < 0.15, (_losses(full), _losses(resumed))


@pytest.mark.parametrize("mp,pp,world,acc,mbs", [(2, 2, 4, 2, 2), (2, 1, 2, 2, 2), (1, 1, 2, 1, 2), (1, 2, 4, 1, 2),
                                                 (2, 2, 8, 1, 2), (1, 1, 4, 1, 1)])
def test_parallel_losses_match_single_rank(tmp_path, mp, pp, world, acc, mbs):
    """One fp32 checkpoint (1 rank), resumed on 1 rank and under a TP/PP/DP layout with the same global
    batch (ZeRO-1 on): every resumed step's loss agrees to 1e-5 relative.  This checks the tensor-parallel
    math and that data-parallel gradients are complete when reduced (overlapped bucket reduction
    included: a bucket reduced before all of its gradients were written would diverge here)."""
    _make_data(tmp_path / "data")
    base = _llama_cfg(tmp_path, 1, 1, 1, acc=2, dropout=False)
    base["topology"]["micro_batch_size"] = 2
    _run(tmp_path, base, 1, "pre")
    out = {}
    dp = world // (mp * pp)
    assert mbs * acc * dp == 4  # same global batch as the reference run
    for key, (m, p, w, a, b) in {"ref": (1, 1, 1, 2, 2), "par": (mp, pp, world, acc, mbs)}.items():
        c = copy.deepcopy(base)
        c["topology"].update(world_size=w, model_parallel_size=m, pipe_parallel_size=p, gradient_accumulation_steps=a,
                             micro_batch_size=b)
        c["trainer"].update(assert_checkpoint_loaded=True, save_dir=None)
        out[key] = _losses(_run(tmp_path, c, w, key))
    np.testing.assert_allclose(out["par"], out["ref"], rtol=1e-5)


def test_mixed_local_global_heads_tp2_matches_single_rank(tmp_path):
    """Heads [0, 2) of 4 windowed, the rest global, split over TP=2 (one partition all local, one all
    global): resumed losses equal the single-rank run to 1e-5 (the reference has no TP support here)."""
    _make_data(tmp_path / "data")
    base = _llama_cfg(tmp_path, 1, 1, 1, acc=2, dropout=False)
    base["transformer_architecture"].update(num_local_attention_heads=2, local_attention_window_size=16,
                                            masked_softmax={"kernel": "flash_attention"})
    _run(tmp_path, base, 1, "pre")
    out = {}
    for key, (m, w) in {"ref": (1, 1), "tp2": (2, 2)}.items():
        c = copy.deepcopy(base)
        c["topology"].update(world_size=w, model_parallel_size=m)
        c["trainer"].update(assert_checkpoint_loaded=True, save_dir=None)
        out[key] = _losses(_run(tmp_path, c, w, key))
    np.testing.assert_allclose(out["tp2"], out["ref"], rtol=1e-5)
