"""End-to-end training on CPU/gloo of a tiny transformer: data pipeline -> 3D-parallel engine -> ZeRO-1
optimizer -> checkpoint at step 6 -> resume must reproduce steps 7-10 exactly (reference:
tests/transformer/test_training.py, which asserts diff_pct < 1e-10 after resume)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from tests.dist_utils import free_port

pytestmark = pytest.mark.cpu
ROOT = Path(__file__).resolve().parent.parent


def _make_data(prefix: Path) -> None:
    sys.path.insert(0, str(ROOT))
    from scaling_amd.core import MemoryMapDatasetBuilder

    rng = np.random.RandomState(0)
    with MemoryMapDatasetBuilder(prefix) as b:
        for _ in range(300):
            b.add(rng.randint(1, 1000, size=rng.randint(10, 300)))


def _config(tmp: Path, mp: int, pp: int, world: int, **arch_over) -> dict:
    topo = {"world_size": world, "model_parallel_size": mp, "pipe_parallel_size": pp, "micro_batch_size": 2,
            "gradient_accumulation_steps": 2, "activation_checkpointing_type": arch_over.pop("checkpointing", "disabled"),
            "sequence_parallel": arch_over.pop("sequence_parallel", False)}
    arch = {"vocab_size": 1024, "sequence_length": 64, "hidden_size": 64, "num_attention_heads": 4, "num_layers": 2,
            "precision": "float32", "dropout_embedding": 0.1, "dropout_attention_probs": 0.1,
            "dropout_after_attention": 0.1, "dropout_after_mlp": 0.1, "masked_softmax": {"kernel": "torch"},
            "norm_type": "rms", "mlp_type": "swiglu", "mlp_factor": 2.0, "weight_tying": False,
            "attention_num_kv_heads": 2, "attention_qkv_in_one": False}
    arch.update(arch_over)
    return {
        "topology": topo,
        "optimizer": {"beta1": 0.9, "beta2": 0.99, "gradient_clipping": 1.0, "zero": True},
        "learning_rate_scheduler": {"learning_rate": 0.01, "learning_rate_warmup_steps": 2,
                                    "learning_rate_decay_iters": 10, "learning_rate_decay_style": "cosine"},
        "embedding_learning_rate_scheduler": {"learning_rate": 0.001, "learning_rate_warmup_steps": 2,
                                              "learning_rate_decay_iters": 10, "learning_rate_decay_style": "cosine"},
        "training": {"use_separate_lr_on_embeddings": True},
        "trainer": {"save_dir": str(tmp / "ckpt"), "save_interval": 6, "load_dir": str(tmp / "ckpt"),
                    "train_iterations": 10, "assert_checkpoint_loaded": False},
        "logger": {"log_level": "warning", "log_dir": str(tmp / "logs")},
        "profiler": {"profile_steps": 2, "profile_start_at_step": 1},
        "data": {"data_prefixes": [str(tmp / "data")], "blended_dataset": {"cache_directory": str(tmp)}},
        "transformer_architecture": arch,
    }


def _run(tmp: Path, cfg: dict, world: int, tag: str) -> list:
    spec = tmp / f"{tag}.json"
    out = tmp / f"{tag}.out.json"
    spec.write_text(json.dumps({"config": cfg, "out": str(out)}))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "tests" / "train_helper.py"), str(spec)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(out.read_text())


@pytest.mark.parametrize(
    "mp,pp,world,extra",
    [
        (1, 1, 1, {}),
        (1, 1, 2, {}),
        (2, 1, 2, {}),
        (1, 2, 2, {}),
        (2, 1, 2, {"sequence_parallel": True}),
        (1, 1, 1, {"checkpointing": "every_layer", "norm_type": "layernorm", "mlp_type": "default", "mlp_factor": 4.0,
                   "weight_tying": True, "attention_num_kv_heads": None, "attention_qkv_in_one": True}),
        (1, 2, 2, {"checkpointing": "every_pipe_stage", "weight_tying": True}),
    ],
)
def test_train_and_resume_bit_exact(tmp_path, mp, pp, world, extra):
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, mp, pp, world, **extra)
    full = _run(tmp_path, cfg, world, "full")
    assert len(full) == 10
    assert all(np.isfinite(m["training/loss"]) for m in full)
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, cfg, world, "resumed")
    assert [m["training/loss"] for m in resumed] == [m["training/loss"] for m in full[-4:]]
    assert (tmp_path / "ckpt" / "global_step6").is_dir()
    # the profiler wrote its timings
    assert any(p.name == "profile.json" for p in (tmp_path / "logs").rglob("profile.json"))


@pytest.mark.parametrize(
    "mp,pp,world,extra",
    [
        (1, 1, 2, {}),
        (2, 1, 2, {}),
        (1, 2, 2, {"weight_tying": True}),
    ],
)
def test_lazy_grad_zeroing_matches_eager(tmp_path, mp, pp, world, extra):
    """Optimizer ``lazy_grad_zeroing`` (no per-step gradient memset; first GEMM-fused weight-gradient write with
    beta = 0, autograd-accumulated grads zeroed by a tensor hook, untouched grads zeroed before the step) must give
    bit-identical losses to eager zeroing, with gradient accumulation, ZeRO, TP and tied weights under PP."""
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, mp, pp, world, **extra)
    cfg["trainer"]["save_dir"] = None
    cfg["trainer"]["load_dir"] = None
    eager = _run(tmp_path, cfg, world, "eager")
    cfg["optimizer"]["lazy_grad_zeroing"] = True
    lazy = _run(tmp_path, cfg, world, "lazy")
    assert [m["training/loss"] for m in lazy] == [m["training/loss"] for m in eager]
    assert [m["training/global_grad_norm"] for m in lazy] == [m["training/global_grad_norm"] for m in eager]


def test_sequence_parallel_dp_overlap_matches_serial(tmp_path):
    """TP2 x DP2 with sequence parallelism: the DP gradient reduction launched bucket by bucket during the backward
    (norm-weight buckets deferred until their TP all-reduce) gives the same losses as reducing everything after it."""
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, 2, 1, 4, sequence_parallel=True)
    cfg["trainer"]["save_dir"] = None
    cfg["trainer"]["load_dir"] = None
    cfg["optimizer"]["grad_bucket_numel"] = 4096  # many buckets: norm weights share buckets with matrices
    cfg["optimizer"]["overlap_grad_reduce"] = False
    serial = _run(tmp_path, cfg, 4, "serial")
    cfg["optimizer"]["overlap_grad_reduce"] = True
    overlap = _run(tmp_path, cfg, 4, "overlap")
    assert [m["training/loss"] for m in overlap] == [m["training/loss"] for m in serial]


def test_async_checkpointing_resume_bit_exact(tmp_path):
    """``trainer.async_checkpointing``: files written by the background writer (host snapshot, .tmp + rename) are the
    same checkpoint: resuming from it reproduces steps 7-10 of an uninterrupted run exactly, and ``latest`` names
    the step once the end-of-training flush has published it."""
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, 1, 2, 2)
    cfg["trainer"]["async_checkpointing"] = True
    full = _run(tmp_path, cfg, 2, "full")
    assert (tmp_path / "ckpt" / "latest").read_text().strip() == "global_step6"
    assert not list((tmp_path / "ckpt").rglob("*.tmp"))
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    cfg["trainer"]["async_checkpointing"] = False
    resumed = _run(tmp_path, cfg, 2, "resumed")
    assert [m["training/loss"] for m in resumed] == [m["training/loss"] for m in full[-4:]]


def test_bf16_gradient_reduction_tracks_fp32(tmp_path):
    """``optimizer.grad_reduce_dtype='bfloat16'`` (bf16 reduce-scatter of the bf16 gradient buckets, then cast and
    1/dp scale into the fp32 owned shard) trains like the fp32 reduction: same step-1 loss, and later losses within
    bf16 rounding of the gradients.  Model in bf16 so the bf16 branch is taken."""
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, 1, 1, 2, precision="bfloat16", dropout_embedding=0.0, dropout_attention_probs=0.0,
                  dropout_after_attention=0.0, dropout_after_mlp=0.0)
    cfg["trainer"]["save_dir"] = None
    cfg["trainer"]["load_dir"] = None
    fp32 = _run(tmp_path, cfg, 2, "fp32")
    cfg["optimizer"]["grad_reduce_dtype"] = "bfloat16"
    bf16 = _run(tmp_path, cfg, 2, "bf16")
    a = np.array([m["training/loss"] for m in fp32])
    b = np.array([m["training/loss"] for m in bf16])
    assert np.all(np.isfinite(b))
    assert a[0] == b[0]
    assert not np.array_equal(a, b)  # the bf16 reduction path ran (different rounding from step 2 on)
    assert np.max(np.abs(a - b) / np.abs(a)) < 2e-2, (a, b)


def test_deterministic_torch_training_cpu(tmp_path):
    """``training.use_deterministic_torch_algorithms: true`` on the CPU path: every op passes torch's check and two
    runs are bit-identical (reference tests/transformer/test_training.py:845-862)."""
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, 1, 1, 1)
    cfg["training"]["use_deterministic_torch_algorithms"] = True
    cfg["trainer"]["save_dir"] = None
    cfg["trainer"]["load_dir"] = None
    a = _run(tmp_path, cfg, 1, "det_a")
    b = _run(tmp_path, cfg, 1, "det_b")
    assert [m["training/loss"] for m in a] == [m["training/loss"] for m in b]


@pytest.mark.parametrize("mp,pp,world", [(1, 1, 1), (2, 1, 2)])
def test_keep_attention_checkpointing_matches_every_layer(tmp_path, mp, pp, world):
    """``activation_checkpointing_type: every_layer_keep_attention`` trains exactly like ``every_layer`` (on CPU the
    attention has no flash kernel to keep, so this pins the mode's plumbing; the GPU test pins the reuse)."""
    _make_data(tmp_path / "data")
    runs = {}
    for ac in ("every_layer", "every_layer_keep_attention", "every_layer_save_matmuls"):
        cfg = _config(tmp_path, mp, pp, world, checkpointing=ac)
        cfg["trainer"]["save_dir"] = None
        cfg["trainer"]["load_dir"] = None
        runs[ac] = [m["training/loss"] for m in _run(tmp_path, cfg, world, ac)]
    assert runs["every_layer"] == runs["every_layer_keep_attention"]
    # selective recompute (GEMM outputs kept, element-wise work recomputed) is the same arithmetic
    assert runs["every_layer"] == runs["every_layer_save_matmuls"]


def test_save_matmuls_checkpointing_skips_gemms_in_recompute():
    """``every_layer_save_matmuls``: the backward's recompute of a checkpointed layer runs no linear-layer GEMM (every
    forward GEMM output is replayed from the first forward), gradients equal plain per-layer checkpointing, and a kept
    output modified in place after the first forward is recomputed instead of replayed."""
    import torch

    import scaling_amd.core.nn.linear.main_grad as mg
    from scaling_amd.core.nn.parallel_module.activation_checkpointing import checkpoint_with_rng
    from scaling_amd.models import llama_architecture
    from scaling_amd.ops.attention import AttentionStash, attention_stash, stash_gemm
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig
    from scaling_amd.transformer.model.layers import TransformerLayer
    from scaling_amd.transformer.model.layers.base import TransformerLayerIO

    torch.manual_seed(0)
    arch = TransformerArchitectureConfig(**llama_architecture("llama_tiny", sequence_length=32, vocab_size=64))
    layer = TransformerLayer(arch, layer_index=0)
    real = mg.gemm_linear
    calls = []

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)

    grads = {}
    for gemms in (False, True):
        calls.clear()
        layer.zero_grad(set_to_none=True)
        dt = next(layer.parameters()).dtype
        x = torch.randn(2, 32, arch.hidden_size, generator=torch.Generator().manual_seed(1)).to(dt).requires_grad_()
        cu = torch.tensor([0, 32, 64], dtype=torch.int32)
        pos = torch.arange(32).unsqueeze(0).expand(2, -1).contiguous()
        io = TransformerLayerIO(activations=x, position_ids=pos, cumulative_seq_lengths_padded=cu,
                                cumulative_seq_lengths=cu)
        mg.gemm_linear = counting
        try:
            out = checkpoint_with_rng(layer._forward_tuple_input, None, True, *layer.input_to_tuple(io),
                                      keep_gemms=gemms)
            n_fwd = len(calls)
            out.hidden().pow(2).mean().backward()
        finally:
            mg.gemm_linear = real
        assert n_fwd > 0
        assert len(calls) == (n_fwd if gemms else 2 * n_fwd), (gemms, n_fwd, len(calls))
        grads[gemms] = [x.grad.clone()] + [p.grad.clone() for p in layer.parameters() if p.grad is not None]
    for a, b in zip(grads[False], grads[True]):
        assert torch.equal(a, b)

    # a kept output changed in place (a LoRA up-projection accumulating into it) is recomputed, not replayed
    stash = AttentionStash(keep_gemms=True)
    with attention_stash(stash, "record"):
        y = stash_gemm(lambda: torch.ones(3))
    y.add_(1)
    with attention_stash(stash, "replay"):
        z = stash_gemm(lambda: torch.full((3,), 7.0))
    assert torch.equal(z, torch.full((3,), 7.0))
    stash = AttentionStash(keep_gemms=True)
    with attention_stash(stash, "record"):
        y = stash_gemm(lambda: torch.ones(3))
    with attention_stash(stash, "replay"):
        z = stash_gemm(lambda: torch.full((3,), 7.0))
    assert torch.equal(z, torch.ones(3))
