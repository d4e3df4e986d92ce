"""LoRA adapters of ParallelSelfAttention on gloo (reference ``tests/core/test_nn/test_lora.py:259-343``)
and a LoRA finetune end-to-end run at DP=2 with ZeRO.

Stricter than the reference (which compares merged/unmerged outputs with atol=1e6): merged and unmerged
outputs agree to 1e-4 in fp32; under TP=2 every rank's ``get_delta_weights`` equals its shard of
``scaling * B @ A`` built from the all-gathered adapter weights; the merge removes the adapters and
changes exactly the targeted projections.
"""
from __future__ import annotations

from pathlib import Path

import pytest
import torch

from tests.dist_utils import make_topology, run_distributed

pytestmark = pytest.mark.cpu

CASES = [(mp, kv, one) for mp in (1, 2) for kv in (None, 2) for one in (True, False) if not (kv and one)]
MODULES = [["query"], ["value", "dense"], ["query", "key"], ["query", "key", "value", "dense"]]


def _gather(t: torch.Tensor, dim: int, topo) -> torch.Tensor:
    import torch.distributed as dist

    n = topo.config.model_parallel_size
    if n == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(n)]
    dist.all_gather(parts, t.contiguous(), group=topo.model_parallel_group)
    return torch.cat(parts, dim=dim)


def _lora_case(mp: int, kv, qkv_in_one: bool, modules: list, rank: int):
    import torch.distributed as dist

    from scaling_amd.core import LoRaConfig, LoRAModuleType, MaskedSoftmaxConfig, ParallelSelfAttention
    from scaling_amd.core.nn.attention.attention import RelativePositionEmbeddingType

    topo = make_topology(model_parallel_size=mp, micro_batch_size=1)
    torch.manual_seed(1234)
    cfg = LoRaConfig.from_dict({"parallel_modules": modules, "rank": rank, "alpha": 4})
    attn = ParallelSelfAttention(hidden_size=256, num_attention_heads=4, num_kv_heads=kv, qkv_in_one=qkv_in_one,
                                 lora_config=cfg, topology=topo, masked_softmax_config=MaskedSoftmaxConfig(),
                                 relative_position_embedding_type=RelativePositionEmbeddingType.NONE)
    assert len(attn.lora_modules) == len(modules)
    torch.manual_seed(99 + topo.model_parallel_rank)
    with torch.no_grad():
        for mod in attn.lora_modules.values():  # B is zero-initialised: make the adapters visible
            mod.dense_out.weight.copy_(torch.rand_like(mod.dense_out.weight) * 0.1)

    # get_delta_weights is this rank's shard of scaling * B @ A over the full adapter
    for name, mod in attn.lora_modules.items():
        dense = mod.lora_module_type == LoRAModuleType.DENSE
        a_full = _gather(mod.dense_in.weight.detach(), 0, topo)
        b_full = _gather(mod.dense_out.weight.detach(), 1 if dense else 0, topo)
        full = (b_full @ a_full) * mod.scaling
        n, r = mp, topo.model_parallel_rank
        shard = full.chunk(n, dim=1 if dense else 0)[r]
        torch.testing.assert_close(mod.get_delta_weights(), shard, rtol=1e-5, atol=1e-6, msg=name)

    torch.manual_seed(7)
    b, s = 3, 16
    x = torch.randn(b, s, 256)
    cu = torch.arange(0, (b + 1) * s, s, dtype=torch.int32)
    pos = torch.arange(s).repeat(b, 1)
    with torch.no_grad():
        y0 = attn(x, cumulative_seq_lengths=cu, position_ids=pos)
    assert y0.shape == (b, s, 256)

    targets = ["query_key_value"] if qkv_in_one else [m for m in modules if m != "dense"]
    if "dense" in modules:
        targets.append("dense")
    before = {t: getattr(attn, t).weight.detach().clone() for t in targets}
    untouched = [t for t in ("query", "key", "value") if not qkv_in_one and t not in modules]
    before_untouched = {t: getattr(attn, t).weight.detach().clone() for t in untouched}
    attn.merge_lora_weights()
    assert not hasattr(attn, "lora_modules") and attn.lora_merged_state is True
    for t, w in before.items():
        assert not torch.equal(w, getattr(attn, t).weight), f"{t} unchanged after merge"
    for t, w in before_untouched.items():
        assert torch.equal(w, getattr(attn, t).weight), f"{t} changed by merge"
    with torch.no_grad():
        y1 = attn(x, cumulative_seq_lengths=cu, position_ids=pos)
    torch.testing.assert_close(y1, y0, rtol=1e-4, atol=1e-4)
    assert dist.get_world_size() == mp
    return True


@pytest.mark.parametrize("mp,kv,qkv_in_one", CASES)
@pytest.mark.parametrize("modules", MODULES)
@pytest.mark.parametrize("rank", [4, 16])
def test_lora_forward_merge_equal(mp, kv, qkv_in_one, modules, rank):
    assert all(run_distributed(_lora_case, mp, mp=mp, kv=kv, qkv_in_one=qkv_in_one, modules=modules,
                               rank=rank).values())


def test_lora_finetune_dp2_zero(tmp_path: Path):
    """Pretrain a tiny Llama-style model, then finetune only LoRA adapters at DP=2 with ZeRO-1: adapter
    weights move, every base weight of the checkpoint stays bit-identical."""
    from tests.test_finetuning import _compare
    from tests.test_training import _config, _make_data, _run

    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, 1, 1, 2, relative_position_embedding_type="rotary_complex")
    cfg["topology"]["gradient_accumulation_steps"] = 1
    _run(tmp_path, cfg, 2, "pre")
    cfg["trainer"].update(assert_checkpoint_loaded=True, load_optimizer_states=False, load_context=False,
                          save_interval=2, train_iterations=4, allowed_missing_keys_in_checkpoint=["lora"])
    cfg["training"].update(finetune=True, finetunable_parameters=["lora"], use_separate_lr_on_embeddings=False)
    cfg["transformer_architecture"]["lora_config"] = {"name": "lora", "rank": 8, "alpha": 16,
                                                      "parallel_modules": ["query", "key", "value", "dense"]}
    # non-zero B after the first update needs a few steps: compare step 2 vs step 4
    ft = _run(tmp_path, cfg, 2, "ft")
    assert len(ft) == 4
    assert _compare(tmp_path, "lora", layer_filter="TransformerLayer") > 0


def _in_base_case(modules, kv, device: str, dtype: torch.dtype, kernel: str, rtol: float, atol: float):
    from scaling_amd.core import LoRaConfig, MaskedSoftmaxConfig, ParallelSelfAttention
    from scaling_amd.core.nn.attention.attention import RelativePositionEmbeddingType
    from scaling_amd.core.nn.rotary_config import RotaryConfig

    torch.manual_seed(1234)
    cfg = LoRaConfig.from_dict({"parallel_modules": modules, "rank": 8, "alpha": 3})
    attn = ParallelSelfAttention(hidden_size=128, num_attention_heads=4, num_kv_heads=kv, qkv_in_one=False, bias=False,
                                 lora_config=cfg, masked_softmax_config=MaskedSoftmaxConfig(kernel=kernel),
                                 relative_position_embedding_type=RelativePositionEmbeddingType.ROTARY,
                                 rotary_config=RotaryConfig(dimensions=32, max_seq_length=64), dtype=dtype,
                                 device=torch.device(device))
    with torch.no_grad():
        for mod in attn.lora_modules.values():
            mod.dense_out.weight.copy_(torch.rand_like(mod.dense_out.weight) * 0.1)
    b, s = 2, 64
    x0 = torch.randn(b, s, 128, device=device, dtype=dtype)
    cu = torch.arange(0, (b + 1) * s, s, dtype=torch.int32, device=device)
    pos = torch.arange(s, device=device).repeat(b, 1)
    lora_params = [p for n, p in attn.named_parameters() if "lora" in n]
    wgt = torch.linspace(-1, 1, x0.numel(), device=device, dtype=dtype).view_as(x0)

    def run(in_base: bool):
        x = x0.clone().requires_grad_(True)
        calls = []
        orig = attn._lora_into_base

        def spy(xx, base):
            r = orig(xx, base) if in_base else False
            calls.append(r)
            return r

        attn._lora_into_base = spy
        if not in_base:  # the unfused reference: no adapter accumulates into a GEMM output (dense included)
            attn._lora_gemm_accumulates = lambda m: False
        try:
            y = attn(x, cumulative_seq_lengths=cu, position_ids=pos)
        finally:
            del attn._lora_into_base
            attn.__dict__.pop("_lora_gemm_accumulates", None)
        assert calls == [in_base]
        grads = torch.autograd.grad((y * wgt).sum(), [x, *lora_params])
        return y.detach().float(), [g.float() for g in grads]

    y_a, g_a = run(True)
    y_b, g_b = run(False)
    torch.testing.assert_close(y_a, y_b, rtol=rtol, atol=atol)
    for ga, gb in zip(g_a, g_b):
        torch.testing.assert_close(ga, gb, rtol=rtol, atol=atol * max(1.0, gb.abs().max().item()))


IN_BASE_MODULES = [["query", "key", "value", "dense"], ["key"], ["query", "value"]]


@pytest.mark.parametrize("modules", IN_BASE_MODULES)
@pytest.mark.parametrize("kv", [None, 2])
def test_lora_in_base_matches_separate_adds(modules, kv):
    """The single-GEMM q/k/v adapter path (A matrices concatenated, scaled up-projections accumulated by the GEMM
    into the base q/k/v output; the dense adapter likewise into the dense output) computes the same outputs and
    gradients as adapter-by-adapter additions."""
    _in_base_case(modules, kv, "cpu", torch.float32, "torch", 1e-5, 1e-5)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("modules", IN_BASE_MODULES)
@pytest.mark.parametrize("kv", [None, 2])
def test_lora_in_base_fused_rope_flash_gpu(modules, kv):
    """On MI355X the in-base adapters feed the fused RoPE + flash-attention node (HIP kernels); the reference
    is the unfused path (adapter additions, separate RoPE, flash attention) in bf16."""
    _in_base_case(modules, kv, "cuda", torch.bfloat16, "flash_attention", 2e-2, 2e-2)
