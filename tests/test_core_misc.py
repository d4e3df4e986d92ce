"""Config / topology / pipeline schedule / runner / numerics of CPU reference paths.
(Reference: tests/core/test_config, test_topology, test_nn/test_pipeline_schedule.py, test_rotary.py,
test_runner, test_pipe_communication.py.)"""
import json
from pathlib import Path

import pytest
import torch

from tests.dist_utils import make_topology, run_distributed

pytestmark = pytest.mark.cpu
REF = Path("/root/reference")


# ---------------------------------------------------------------- config
def test_base_config_frozen_forbid_and_overwrite(tmp_path):
    from pydantic import ValidationError

    from scaling_amd.core import TopologyConfig
    from scaling_amd.core.config.base import overwrite_recursive

    cfg = TopologyConfig(global_rank=0, world_size=8, model_parallel_size=2, pipe_parallel_size=2,
                         global_batch_size=16, micro_batch_size=2)
    assert cfg.data_parallel_size == 2 and cfg.gradient_accumulation_steps == 4
    with pytest.raises(ValidationError):
        TopologyConfig(world_size=8, model_parallel_size=2, pipe_parallel_size=2, global_batch_size=16,
                       micro_batch_size=2, not_a_field=1)
    with pytest.raises(Exception):
        cfg.world_size = 4  # frozen
    d = {"a": {"b": 1, "c": 2}}
    overwrite_recursive(d, {"a": {"c": 3}, "x": 1})
    assert d == {"a": {"b": 1, "c": 3}, "x": 1}


@pytest.mark.parametrize("inp,expect", [
    (dict(world_size=16, model_parallel_size=2, pipe_parallel_size=4, global_batch_size=32, gradient_accumulation_steps=2),
     dict(data_parallel_size=2, micro_batch_size=8)),
    (dict(world_size=1, model_parallel_size=1, pipe_parallel_size=1, global_batch_size=16, gradient_accumulation_steps=1),
     dict(data_parallel_size=1, micro_batch_size=16)),
    (dict(model_parallel_size=2, pipe_parallel_size=2, data_parallel_size=2, micro_batch_size=2, gradient_accumulation_steps=3),
     dict(world_size=8, global_batch_size=12)),
])
def test_topology_config_inference(inp, expect):
    from scaling_amd.core import TopologyConfig

    cfg = TopologyConfig(global_rank=0, **inp)
    for k, v in expect.items():
        assert getattr(cfg, k) == v


def test_topology_config_rejects_inconsistent_batch():
    from scaling_amd.core import TopologyConfig

    with pytest.raises(Exception):
        TopologyConfig(global_rank=0, world_size=4, model_parallel_size=1, pipe_parallel_size=1, global_batch_size=10,
                       micro_batch_size=4, gradient_accumulation_steps=1)


@pytest.mark.skipif(not (REF / "examples/transformer_example/config.yml").exists(), reason="reference not mounted")
def test_reference_transformer_config_loads_unchanged():
    from scaling_amd.transformer import TransformerConfig

    cfg = TransformerConfig.from_yaml(REF / "examples/transformer_example/config.yml")
    assert cfg.transformer_architecture.hidden_size == 256
    again = TransformerConfig.from_dict(json.loads(json.dumps(cfg.as_dict())))
    a, b = again.as_dict(), cfg.as_dict()
    a.pop("logger"), b.pop("logger")  # logger validation appends a timestamp to the wandb group
    assert a == b


def test_config_template_roundtrip(tmp_path):
    from scaling_amd.transformer import TransformerConfig

    p = tmp_path / "template.yml"
    TransformerConfig.save_template(p)
    text = p.read_text()
    assert "transformer_architecture" in text and "#" in text


# ---------------------------------------------------------------- topology grid (4 ranks, gloo)
def _grid_case():
    topo = make_topology(model_parallel_size=2, pipe_parallel_size=2)
    r = topo.config.global_rank
    # rank grid arange(world).reshape(pp, dp, mp): mp innermost, then dp, then pp
    pp, dp, mp = r // 2, 0, r % 2
    assert (topo.pipe_parallel_rank, topo.data_parallel_rank, topo.model_parallel_rank) == (pp, dp, mp)
    assert topo.get_global_rank(pipe_parallel_rank=pp, data_parallel_rank=dp, model_parallel_rank=mp) == r
    assert topo.is_first_pipe_parallel_rank == (pp == 0) and topo.is_last_pipe_parallel_rank == (pp == 1)
    assert topo.is_io_rank == (mp == 0)
    return True


def test_topology_rank_grid_world4():
    assert all(run_distributed(_grid_case, 4).values())


# ---------------------------------------------------------------- pipeline schedule
@pytest.mark.parametrize("pp", [1, 2, 7])
@pytest.mark.parametrize("acc", [1, 2, 7, 16])
def test_train_schedule_is_complete(pp, acc):
    from scaling_amd.core.nn.pipeline_schedule.instructions import (InstructionBackwardPass, InstructionForwardPass,
                                                                    InstructionOptimizerStep)
    from scaling_amd.core.nn.pipeline_schedule.train import PipelineScheduleTrain

    class T:
        def __init__(self, stage):
            from scaling_amd.core import TopologyConfig

            self.config = TopologyConfig(global_rank=0, world_size=pp, model_parallel_size=1, pipe_parallel_size=pp,
                                         micro_batch_size=1, gradient_accumulation_steps=acc)
            self.pipe_parallel_rank = stage
            self.is_first_pipe_parallel_rank = stage == 0
            self.is_last_pipe_parallel_rank = stage == pp - 1
            self.previous_pipe_parallel_rank = stage - 1 if stage > 0 else None
            self.next_pipe_parallel_rank = stage + 1 if stage < pp - 1 else None

    for stage in range(pp):
        ins = PipelineScheduleTrain(topology=T(stage)).instructions()
        fwd = sorted(i.micro_batch_id for i in ins if isinstance(i, InstructionForwardPass))
        bwd = sorted(i.micro_batch_id for i in ins if isinstance(i, InstructionBackwardPass))
        assert fwd == list(range(acc)) and bwd == list(range(acc))
        assert isinstance(ins[-1], InstructionOptimizerStep)


def test_schedule_visualize(tmp_path):
    from scaling_amd.core import PipelineScheduleInference, PipelineScheduleTrain

    img = PipelineScheduleTrain.visualize(gradient_accumulation_steps=4, pipe_parallel_size=3)
    img.save(tmp_path / "train.png")
    PipelineScheduleInference.visualize(gradient_accumulation_steps=1, pipe_parallel_size=3).save(tmp_path / "inf.png")
    assert (tmp_path / "train.png").stat().st_size > 0


# ---------------------------------------------------------------- runner
def test_runner_host_parsing_and_payload():
    from scaling_amd.core.runner.launch_config import decode_base64
    from scaling_amd.core.runner.runner import encode_base64, parse_host

    assert parse_host("node-1 slots=0,2,3", 8) == ("node-1", [0, 2, 3])
    assert parse_host("node-2 slots=4", 8) == ("node-2", [0, 1, 2, 3])
    assert parse_host("node-3", 2) == ("node-3", [0, 1])
    d = {"a": [1, 2], "b": {"c": "x"}}
    assert decode_base64(encode_base64(d)) == d


# ---------------------------------------------------------------- numerics (CPU reference paths)
def test_rotary_tokens_matches_reference_forward():
    from scaling_amd.core import RotaryConfig
    from scaling_amd.core.nn.rotary import RotaryEmbedding, RotaryEmbeddingComplex

    torch.manual_seed(0)
    for cls in (RotaryEmbedding, RotaryEmbeddingComplex):
        rot = cls(RotaryConfig(dimensions=16, max_seq_length=64, base=10000), device=torch.device("cpu"))
        x = torch.randn(2 * 8, 4, 16)
        pos = torch.arange(8).repeat(2)
        y = rot.apply_tokens(x, pos, 8)
        # rotation preserves pair norms and is undone by the inverse position
        assert torch.allclose(y.norm(dim=-1), x.norm(dim=-1), atol=1e-5)
        assert torch.allclose(y[:1], x[:1], atol=1e-6)  # position 0 is the identity


def test_norms_match_torch():
    from scaling_amd.ops.norm import layer_norm, rms_norm

    torch.manual_seed(0)
    x = torch.randn(5, 64, requires_grad=True)
    w = torch.randn(64, requires_grad=True)
    b = torch.randn(64, requires_grad=True)
    y = layer_norm(x, w, b, 1e-5)
    torch.testing.assert_close(y, torch.nn.functional.layer_norm(x, (64,), w, b, 1e-5))
    r = rms_norm(x, w, 1e-5)
    torch.testing.assert_close(r, x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * w)


def test_lora_merge_equivalence():
    from scaling_amd.core import MaskedSoftmaxConfig, ParallelSelfAttention, RotaryConfig
    from scaling_amd.core.nn.lora_config import LoRaConfig

    torch.manual_seed(0)
    attn = ParallelSelfAttention(hidden_size=32, num_attention_heads=4, masked_softmax_config=MaskedSoftmaxConfig(),
                                 lora_config=LoRaConfig(rank=4, alpha=8), device=torch.device("cpu"), bias=False,
                                 rotary_config=RotaryConfig(dimensions=8, max_seq_length=16, base=10000))
    for n, p in attn.named_parameters():
        if "lora" in n:
            torch.nn.init.normal_(p, std=0.1)
    x = torch.randn(2, 6, 32)
    cu = torch.tensor([0, 6, 12], dtype=torch.int32)
    pos = torch.arange(6).repeat(2, 1)
    with torch.no_grad():
        y1 = attn(x, cumulative_seq_lengths=cu, position_ids=pos)
        attn.merge_lora_weights()
        y2 = attn(x, cumulative_seq_lengths=cu, position_ids=pos)
    torch.testing.assert_close(y1, y2, rtol=1e-4, atol=1e-5)


def test_flash_dropout_mask_twin_matches_integer_reference():
    """ops.attention.dropout_keep_mask (the PyTorch twin of the fused kernel mask) against plain Python
    uint32 arithmetic of the same hash; keep rate = 1 - p."""
    from scaling_amd.ops import attention as A

    M = 0xFFFFFFFF

    def mix(x):
        x ^= x >> 16
        x = (x * 0x7FEB352D) & M
        x ^= x >> 15
        x = (x * 0x846CA68B) & M
        return x ^ (x >> 16)

    def keep(seed, h, q, k, p):
        row = mix((mix(seed ^ ((h * 0x9E3779B9) & M)) + q) & M)
        return mix(row ^ ((k * 0x85EBCA6B) & M)) >= A.dropout_threshold(p)

    m = A.dropout_keep_mask(123456789, torch.arange(3), torch.arange(50, 66), torch.arange(100, 132), 0.3)
    assert all(bool(m[h, i, j]) == keep(123456789, h, 50 + i, 100 + j, 0.3)
               for h in range(3) for i in range(16) for j in range(32))
    big = A.dropout_keep_mask(7, torch.arange(2), torch.arange(512), torch.arange(512), 0.1)
    assert abs(big.float().mean().item() - 0.9) < 0.01


def test_elementwise_cpu_paths_match_torch():
    from scaling_amd.core.nn.activation_function import ActivationFunction, get_activation_function
    from scaling_amd.ops import elementwise

    x = torch.randn(100)
    torch.testing.assert_close(get_activation_function(ActivationFunction.GELU)(x), torch.nn.functional.gelu(x))
    torch.testing.assert_close(get_activation_function(ActivationFunction.SILU)(x), torch.nn.functional.silu(x))
    assert torch.equal(elementwise.dropout_add(x, x, 0.5, training=False), x + x)
    torch.manual_seed(0)
    a = elementwise.dropout_add(x, None, 0.5, training=True)
    torch.manual_seed(0)
    assert torch.equal(a, torch.nn.functional.dropout(x, 0.5, training=True))


def test_attention_reference_mixed_local_global_heads_matches_two_calls():
    """CPU oracle: per-head window (heads [0, nl) local) equals the reference's two-call split."""
    from scaling_amd.ops.attention import attention_reference

    torch.manual_seed(0)
    T, Hq, Hk, D, nl, w = 40, 6, 2, 16, 2, 5
    q, k, v = torch.randn(T, Hq, D), torch.randn(T, Hk, D), torch.randn(T, Hk, D)
    cu = torch.tensor([0, 25, 40], dtype=torch.int32)
    both = attention_reference(q, k, v, cu, cu, 0.25, True, w, local_heads=nl)
    kr, vr = k.repeat_interleave(Hq // Hk, 1), v.repeat_interleave(Hq // Hk, 1)
    loc = attention_reference(q[:, :nl], kr[:, :nl], vr[:, :nl], cu, cu, 0.25, True, w)
    glob = attention_reference(q[:, nl:], kr[:, nl:], vr[:, nl:], cu, cu, 0.25, True, -1)
    torch.testing.assert_close(both, torch.cat([loc, glob], 1))


def test_async_checkpoint_snapshot_handles_dict_subclasses_and_mutable_leaves():
    """The async writer's host snapshot must accept what a synchronous torch.save accepts (a defaultdict in the
    state) and must not share mutable leaves with the live training state."""
    import collections

    import torch

    from scaling_amd.core.utils.checkpoint_writer import _snapshot

    d = collections.defaultdict(list)
    d["a"].append(torch.ones(2))
    live_set = {1, 2}
    nt = collections.namedtuple("NT", "x y")(torch.zeros(1), 3)
    snap = _snapshot({"d": d, "s": live_set, "nt": nt})
    live_set.add(3)
    d["a"][0].add_(5)
    assert snap["s"] == {1, 2}
    assert torch.equal(snap["d"]["a"][0], torch.ones(2))
    assert type(snap["nt"]).__name__ == "NT" and snap["nt"].y == 3


@pytest.mark.parametrize("pp", [1, 2, 7, 16, 32])
def test_schedule_visualize_grid_and_inference_independent_of_acc(tmp_path, pp):
    """Reference tests/core/test_nn/test_pipeline_schedule.py grid: the train schedule renders for every (pp, acc);
    the inference schedule renders for acc 1 and 2 (acc + pp - 1 steps, so more micro-batches draw wider)."""
    from scaling_amd.core import PipelineScheduleInference, PipelineScheduleTrain

    for acc in (1, 2, 7, 16, 32):
        PipelineScheduleTrain.visualize(gradient_accumulation_steps=acc, pipe_parallel_size=pp)
    a = PipelineScheduleInference.visualize(gradient_accumulation_steps=1, pipe_parallel_size=pp)
    b = PipelineScheduleInference.visualize(gradient_accumulation_steps=2, pipe_parallel_size=pp)
    assert a.size[1] == b.size[1] and b.size[0] > a.size[0]


def test_visualize_measured_profile(tmp_path):
    """A profile written by the framework's own profiler (2-stage pipeline training run) replays through the
    schedule simulator (reference test_visualize_train_profile): per-stage busy / idle times and an image."""
    import json

    from scaling_amd.core import PipelineScheduleTrain
    from tests.test_training import _config, _make_data, _run

    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, 1, 2, 2)
    cfg["trainer"]["save_dir"] = None
    cfg["trainer"]["load_dir"] = None
    cfg["trainer"]["train_iterations"] = 3
    _run(tmp_path, cfg, 2, "prof")
    prof = next((tmp_path / "logs").rglob("profile.json"))
    d = json.loads(prof.read_text())
    assert d["pipe_parallel_size"] == 2 and d["observations"]
    timings, image = PipelineScheduleTrain.visualize_profile(profile_file=prof, milliseconds_per_pixel=0.01,
                                                             pipe_pixels=50)
    assert timings["total_time"] > 0
    assert all(0.0 <= v < 1.0 for v in timings["pct_idling"].values())
    image.save(str(tmp_path / "profile.png"))
