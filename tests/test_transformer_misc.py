"""Transformer suite pieces: inference (cached == uncached generation, samplers, checkpoint round trip),
tokenizer, FLOP accounting, embedding head, image encoder, determined hparam mapping, MLP example.
(Reference: tests/transformer/test_inference.py, test_tokenizer, test_utils.py.)"""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.cpu
REF = Path("/root/reference/tests/transformer/files")
ROOT = Path(__file__).resolve().parent.parent


def _arch(**kw):
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig

    d = dict(vocab_size=128, hidden_size=64, num_layers=2, num_attention_heads=4, sequence_length=64, norm_type="rms",
             mlp_type="swiglu", mlp_factor=2.0, precision="float32", attention_num_kv_heads=2,
             attention_qkv_in_one=False, weight_tying=False, relative_position_embedding_type="rotary_complex")
    d.update(kw)
    return TransformerArchitectureConfig(**d)


@pytest.mark.parametrize("kw", [{}, {"weight_tying": True, "norm_type": "layernorm", "mlp_type": "default",
                                     "mlp_factor": 4.0, "attention_num_kv_heads": None, "attention_qkv_in_one": True,
                                     "relative_position_embedding_type": "rotary"}])
def test_generation_cached_equals_uncached(kw):
    from scaling_amd.transformer.inference import TransformerInferenceModule
    from scaling_amd.transformer.model.model import get_transformer_layer_specs

    torch.manual_seed(0)
    m = TransformerInferenceModule(get_transformer_layer_specs(_arch(**kw)), devices=("cpu",))
    a = m.generate(8, input_tokens=[1, 2, 3, 4, 5], stop_tokens=[127], use_cache=True)
    b = m.generate(8, input_tokens=[1, 2, 3, 4, 5], stop_tokens=[127], use_cache=False)
    assert a.completion_tokens == b.completion_tokens
    torch.testing.assert_close(a.completion_logits, b.completion_logits, rtol=1e-4, atol=1e-4)
    logits = m.logits(input_tokens=[1, 2, 3])
    assert logits.shape == (3, 128)


def test_samplers():
    from scaling_amd.transformer.inference import sample_argmax, sample_temperature, top_k_transform, top_p_transform

    torch.manual_seed(0)
    logits = torch.randn(1, 3, 50)
    assert sample_argmax(logits).item() == logits[0, -1].argmax().item()
    assert 0 <= sample_temperature(logits, 0.7).item() < 50
    k = top_k_transform(logits[0, -1], 5)
    assert torch.isfinite(k).sum() == 5
    p = top_p_transform(logits[0, -1], 0.5)
    assert 1 <= torch.isfinite(p).sum() < 50


@pytest.mark.skipif(not (REF / "llama2-tokenizer.json").exists(), reason="reference tokenizer not mounted")
def test_tokenizer_roundtrip_and_no_prefix_variant():
    from scaling_amd.transformer.tokenizer import load_tokenizers

    tok, tok_nps = load_tokenizers(REF / "llama2-tokenizer.json")
    assert len(tok) == 32000 and tok.eos_token_id == 2
    ids = tok.encode("Hello world")
    assert tok.decode(ids).strip() == "Hello world"
    assert tok_nps.encode("Hello")[0] != tok.encode("Hello")[0]  # no leading-space variant


def test_flop_accounting():
    from scaling_amd.core import TopologyConfig
    from scaling_amd.transformer.utils.get_tflops import (get_model_flop_utilization_palm, get_tflops_aleph_alpha,
                                                          get_tflops_bloom, get_tflops_electra, get_tflops_megatron)

    class T:
        config = TopologyConfig(global_rank=0, world_size=8, model_parallel_size=1, pipe_parallel_size=1,
                                micro_batch_size=4, gradient_accumulation_steps=2)

    a = _arch(hidden_size=4096, num_layers=32, num_attention_heads=32, vocab_size=32000, sequence_length=4096,
              attention_num_kv_heads=None, attention_qkv_in_one=True)
    for f in (get_tflops_aleph_alpha, get_tflops_electra, get_tflops_bloom):
        assert f(1.0, T, a) > 0
    mega = get_tflops_megatron(6_700_000_000, 1.0, T, a)
    # 6 N tokens + attention; tokens = gbs * seq
    tokens = 64 * 4096
    assert abs(mega - (6 * 6.7e9 * tokens + tokens * 4096 * 4096 * 32 * 60) / 8e12) / mega < 1e-9
    assert get_model_flop_utilization_palm(1.0, 6_700_000_000, T, a) >= 0.0


def test_embedding_head_pooling():
    from scaling_amd.transformer.model.layers import TransformerEmbeddingHead

    e = torch.randn(2, 5, 8)
    w = torch.tensor([[1, 1, 0, 0, 0], [0, 0, 0, 0, 0]], dtype=torch.float)
    out = TransformerEmbeddingHead.weighted_mean_pooling(e, w)
    ref0 = (e[0, 0] * 1 + e[0, 1] * 2) / 3
    torch.testing.assert_close(out[0], ref0)


def test_image_encoder_token_shape():
    from scaling_amd.transformer.model.image_encoder import ClipModifiedResNet, clip_transform

    torch.manual_seed(0)
    net = ClipModifiedResNet(layers=[1, 1, 1, 1], num_init_channels=8).eval()
    with torch.no_grad():
        tok = net(torch.randn(1, 3, 96, 96))
    assert tok.shape == (1, 9, 8 * 8 * 4)  # 96/32 = 3 -> 9 tokens, width 8*8*4
    from PIL import Image

    t = clip_transform((32, 32))(Image.new("RGB", (40, 50), (255, 0, 0)))
    assert t.shape == (3, 32, 32)


def test_determined_hparams_mapping():
    from scaling_amd.transformer.train_determined import hparams_to_overrides

    o = hparams_to_overrides({"layout": {"global_batch_size": 8, "sequence_length": 64, "target_train_tokens": 5120,
                                         "warmup_tokens": 512, "model_parallel_size": 2, "kernel": "torch"}})
    assert o["trainer"]["train_iterations"] == 10
    assert o["learning_rate_scheduler"]["learning_rate_warmup_steps"] == 1
    assert o["topology"]["model_parallel_size"] == 2
    assert o["transformer_architecture"]["masked_softmax"] == {"kernel": "torch"}


def test_mlp_example_trains(tmp_path):
    cfg = (ROOT / "examples/mlp_example/config.yml").read_text()
    cfg = cfg.replace('"train_iterations": 50', '"train_iterations": 30').replace('"master_port": 29511', '"master_port": 29641')
    cfg = cfg.replace('"save_dir": ".checkpoints_mlp"', f'"save_dir": "{tmp_path}/ck"')
    cfg = cfg.replace('"log_dir": "debug_logs"', f'"log_dir": "{tmp_path}/logs"')
    (tmp_path / "c.yml").write_text(cfg)
    r = subprocess.run([sys.executable, "-m", "examples.mlp_example.run", str(tmp_path / "c.yml")], cwd=str(ROOT),
                       capture_output=True, text=True, timeout=600, env=dict(os.environ, PYTHONPATH=str(ROOT)))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "completed step 30" in r.stdout + r.stderr


def test_kv_cache_preallocated_growth():
    """The decode cache appends in place and doubles capacity only when full (no per-token concat)."""
    from scaling_amd.core.nn.attention import KVCache

    k0, v0 = torch.randn(5, 2, 4), torch.randn(5, 2, 4)
    c = KVCache.start(k0, v0, headroom=3)
    ref_k, ref_v = [k0], [v0]
    buf = c.k
    for i in range(10):
        k1, v1 = torch.randn(1, 2, 4), torch.randn(1, 2, 4)
        ref_k.append(k1)
        ref_v.append(v1)
        k, v = c.append(k1, v1)
        if i < 3:
            assert c.k is buf  # filled in place while capacity lasts
        assert torch.equal(k, torch.cat(ref_k)) and torch.equal(v, torch.cat(ref_v))
    assert c.length == 15 and c.k.shape[0] >= 15


def test_llama2_7b_example_config_matches_bench_architecture():
    """examples/llama2_7b/config.yml trains exactly the architecture bench.py measures."""
    from pathlib import Path

    from scaling_amd.models import llama_architecture
    from scaling_amd.transformer import TransformerConfig

    root = Path(__file__).resolve().parent.parent
    cfg = TransformerConfig.from_yaml(root / "examples" / "llama2_7b" / "config.yml")
    arch = cfg.transformer_architecture
    for k, v in llama_architecture("llama2_7b", sequence_length=4096).items():
        got = getattr(arch, k)
        got = got.value if hasattr(got, "value") else got
        if isinstance(v, dict):
            continue
        assert got == v, (k, got, v)
    assert cfg.topology.micro_batch_size * cfg.topology.gradient_accumulation_steps == 8


def test_comm_volume_estimate_by_layout():
    """Hand-computed volumes: TP2 (4 all-reduces of [M, h] per layer + the embedding's), PP2 boundary
    activations, DP ZeRO-1 reduce-scatter (fp32) + all-gather (bf16) of the rank's shard."""
    from scaling_amd.transformer.utils.comm_estimate import comm_volume_estimate

    h, L, s, mb, acc = 4096, 32, 4096, 2, 4
    M = mb * s
    e = comm_volume_estimate(hidden_size=h, num_layers=L, seq_len=s, micro_batch=mb, grad_acc=acc, tp=2, pp=1, dp=4,
                             params_per_rank=3_000_000_000)
    assert e["tp_bytes"] == int((4 * 32 + 1) * 1.0 * M * h * 2 * acc)
    assert e["pp_bytes"] == 0
    assert e["dp_bytes"] == int(0.75 * 3e9 * 4 + 0.75 * 3e9 * 2)
    e2 = comm_volume_estimate(hidden_size=h, num_layers=L, seq_len=s, micro_batch=mb, grad_acc=acc, tp=2, pp=2, dp=2,
                              params_per_rank=1_500_000_000)
    assert e2["tp_bytes"] == int((4 * 16 + 1) * 1.0 * M * h * 2 * acc)
    assert e2["pp_bytes"] == 2 * M * h * 2 * acc
    assert e2["dp_ms"] > 0 and e2["tp_ms"] > 0
    e1 = comm_volume_estimate(hidden_size=h, num_layers=L, seq_len=s, micro_batch=8, grad_acc=1, tp=1, pp=1, dp=1,
                              params_per_rank=6_000_000_000)
    assert (e1["tp_bytes"], e1["pp_bytes"], e1["dp_bytes"]) == (0, 0, 0)


class _StageProbe(torch.nn.Module):
    """Layer stub recording whether the partitioner marked it as the output layer of a pipeline stage."""

    def __init__(self) -> None:
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(1))
        self.stage_output = False

    def set_stage_output(self, last_of_stage: bool) -> None:
        self.stage_output = last_of_stage


def test_partitioner_marks_stage_output_layers():
    """a transformer layer that leaves its MLP residual add pending (residual_branch) must not do so when its
    output crosses a pipeline stage (p2p would move two tensors): the partitioner marks the last layer of every stage
    that feeds another stage, and only those."""
    from scaling_amd.core.nn.parallel_module.layer_spec import LayerSpec
    from scaling_amd.core.nn.parallel_module.partitioned_module import PipePartitionedModule

    specs = [LayerSpec(_StageProbe) for _ in range(7)]
    m = PipePartitionedModule(specs, devices=["cpu", "cpu", "cpu"], pipe_partition_overwrite=[0, 3, 5, 7])
    assert [layer.stage_output for layer in m._layers] == [False, False, True, False, True, False, False]


@pytest.mark.parametrize("ac,defer", [("disabled", True), ("every_pipe_stage", True), ("every_layer", False),
                                      ("every_layer_keep_attention", False), ("every_layer_save_matmuls", False)])
def test_residual_defer_policy(ac, defer):
    """The MLP residual add is handed to the next layer unless every layer input is a checkpoint boundary (the pending
    pair would be saved as two tensors) or the layer is a stage output (set_stage_output)."""
    from types import SimpleNamespace

    from scaling_amd.core.topology.topology_config import ActivationCheckpointingType
    from scaling_amd.models import llama_architecture
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig
    from scaling_amd.transformer.model.layers import TransformerLayer

    arch = TransformerArchitectureConfig(**llama_architecture("llama_tiny", sequence_length=32, vocab_size=64,
                                                              precision="float32"))
    from scaling_amd.transformer.model.layers.layer import _DEFER_RESIDUAL, residual_defer_allowed

    topo = SimpleNamespace(config=SimpleNamespace(activation_checkpointing_type=ActivationCheckpointingType(ac)))
    assert residual_defer_allowed(topo) == (defer and _DEFER_RESIDUAL)
    real = TransformerLayer(arch, 0, None)
    assert real._defer_ok is _DEFER_RESIDUAL
    real.set_stage_output(True)
    assert real._defer_ok is False
