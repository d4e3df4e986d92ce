"""Multimodal finetuning end to end on CPU/gloo (reference tests/transformer/test_training.py:305-478, which trains
with ``image_encoder: True`` and the encoder excluded from training).

Here the image path is exercised for real: synthetic PIL-generated ``.jpg`` prompts go through
``FinetuningTextDataset`` (CLIP transform -> 144 image-token slots per image), the frozen CLIP RN50x16 tower +
projection embeds them in ``EmbeddingInput``, and the model trains at TP1 and TP2:

* steps 5-6 of a run resumed from the step-4 checkpoint reproduce the continuous run bit-exactly (the encoder's
  BatchNorm buffers are part of the checkpoint);
* the image encoder's parameters are bit-identical between the step-4 and step-8 checkpoints (frozen through
  ``training.parameters_exclude``) while the trained embedding moved;
* a TP2 run resumed from the TP1 step-4 checkpoint (layout change: weights split, ZeRO state resharded) continues
  with TP1's losses (the encoder runs replicated on both TP ranks).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from tests.dist_utils import free_port
from tests.test_inference_checkpoint import _tokenizer

pytestmark = pytest.mark.cpu
ROOT = Path(__file__).resolve().parent.parent


def _images_and_data(tmp: Path) -> Path:
    from PIL import Image

    rng = np.random.RandomState(0)
    (tmp / "images").mkdir()
    items = []
    for i, (name, color) in enumerate([("red", (220, 30, 30)), ("green", (30, 200, 40)), ("blue", (20, 40, 230)),
                                       ("gray", (128, 128, 128))]):
        px = np.clip(np.array(color)[None, None, :] + rng.randint(-25, 25, size=(96, 96, 3)), 0, 255).astype(np.uint8)
        Image.fromarray(px).save(tmp / "images" / f"{name}.jpg", quality=90)
        items.append({"prompt": ["what colour is the image", f"images/{name}.jpg", " answer:"],
                      "completion": f" {name}"})
        items.append({"prompt": f"the {name} square", "completion": " is a colour"})
    data = tmp / "finetuning.json"
    data.write_text(json.dumps(items * 4))
    return data


def _config(tmp: Path, mp: int, world: int, iters: int) -> dict:
    return {
        "topology": {"world_size": world, "model_parallel_size": mp, "pipe_parallel_size": 1, "micro_batch_size": 1,
                     "gradient_accumulation_steps": 1},
        "optimizer": {"beta1": 0.9, "beta2": 0.99, "gradient_clipping": 1.0, "zero": True},
        "learning_rate_scheduler": {"learning_rate": 0.01, "learning_rate_warmup_steps": 2,
                                    "learning_rate_decay_iters": 10, "learning_rate_decay_style": "cosine"},
        "training": {"parameters_exclude": ["image_encoder"]},
        "trainer": {"save_dir": str(tmp / "ckpt"), "save_interval": 4, "load_dir": str(tmp / "ckpt"),
                    "train_iterations": iters, "assert_checkpoint_loaded": False},
        "logger": {"log_level": "warning", "log_dir": str(tmp / "logs")},
        "data": {"data_prefixes": [str(tmp / "finetuning.json")], "blended_dataset": {"cache_directory": str(tmp)},
                 "finetuning_dataset": True},
        "transformer_architecture": {
            "vocab_size": 512, "vocab_file": str(tmp / "tok.json"), "sequence_length": 176, "hidden_size": 64,
            "num_attention_heads": 4, "num_layers": 2, "precision": "float32", "dropout_embedding": 0.0,
            "dropout_attention_probs": 0.0, "dropout_after_attention": 0.0, "dropout_after_mlp": 0.0,
            "masked_softmax": {"kernel": "torch"}, "norm_type": "rms", "mlp_type": "swiglu", "mlp_factor": 2.0,
            "weight_tying": False, "image_encoder": True,
        },
    }


def _run(tmp: Path, cfg: dict, world: int, tag: str) -> list:
    spec = tmp / f"{tag}.json"
    out = tmp / f"{tag}.out.json"
    spec.write_text(json.dumps({"config": cfg, "out": str(out)}))
    env = dict(os.environ, OMP_NUM_THREADS=str(max(1, (os.cpu_count() or 2) // world // 2)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "tests" / "train_helper.py"),
           str(spec)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=1200)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(out.read_text())


def _layer0(ckpt: Path) -> dict:
    from scaling_amd.core.utils.safe_load import safe_load

    files = sorted(ckpt.glob("model_state_layer_0_*.pt"))
    assert files, f"no layer-0 checkpoint in {ckpt}"
    out: dict = {}
    for f in files:
        out.update(safe_load(f))
    return out


def _train(tmp: Path, mp: int, world: int) -> list:
    tmp.mkdir(parents=True, exist_ok=True)
    _images_and_data(tmp)
    _tokenizer(tmp / "tok.json")
    full = _run(tmp, _config(tmp, mp, world, 6), world, "full")
    assert len(full) == 6 and all(np.isfinite(m["training/loss"]) for m in full)
    cfg = _config(tmp, mp, world, 8)
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp, cfg, world, "resumed")
    assert [m["training/loss"] for m in resumed[:2]] == [m["training/loss"] for m in full[-2:]]
    a, b = _layer0(tmp / "ckpt" / "global_step4"), _layer0(tmp / "ckpt" / "global_step8")
    enc = [k for k in a if "image_encoder" in k and "running_" not in k and "num_batches" not in k]
    assert enc, sorted(a)[:20]
    for k in enc:
        assert torch.equal(a[k], b[k]), f"frozen image-encoder parameter {k} changed"
    emb = [k for k in a if "image_encoder" not in k and "embedding" in k]
    assert emb and any(not torch.equal(a[k], b[k]) for k in emb), "the text embedding did not train"
    return full


def test_multimodal_finetuning_frozen_encoder_tp1_tp2(tmp_path):
    tp1 = _train(tmp_path / "tp1", 1, 1)
    _train(tmp_path / "tp2", 2, 2)
    cfg = _config(tmp_path / "tp1", 2, 2, 6)
    cfg["trainer"].update(load_dir=str(tmp_path / "tp1" / "ckpt" / "global_step4"), save_dir=None,
                          assert_checkpoint_loaded=True)
    cross = _run(tmp_path / "tp1", cfg, 2, "tp2_from_tp1")
    np.testing.assert_allclose([m["training/loss"] for m in cross], [m["training/loss"] for m in tp1[-2:]], rtol=1e-4)
