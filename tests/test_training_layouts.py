"""End-to-end training on CPU/gloo across layout changes and training modes (reference:
tests/core/test_training/test_training.py:238-586 layout-change resume, test_activation_checkpointing.py,
tests/transformer/test_training_sequence_parallel.py, test_load_checkpoint_non_strict.py,
test_training_finetuning_chat.py, test_training_legacy.py, test_training_local_attention.py,
test_backwards_compatibility.py)."""
import copy
from pathlib import Path

import numpy as np
import pytest
import torch

from tests.test_training import _config, _make_data, _run

pytestmark = pytest.mark.cpu
FILES = Path("/root/reference/tests/transformer/files")
needs_fixtures = pytest.mark.skipif(not (FILES / "dataset" / "data.bin").exists(), reason="reference fixtures not mounted")


def _losses(ms):
    return [m["training/loss"] for m in ms]


def _no_dropout(cfg):
    a = cfg["transformer_architecture"]
    for k in ("dropout_embedding", "dropout_attention_probs", "dropout_after_attention", "dropout_after_mlp"):
        a[k] = 0.0
    return cfg


# (mp, pp, world, acc, checkpointing, zero) -> (mp, pp, world, acc, checkpointing, zero); global batch constant
LAYOUT_CHANGES = [
    ((1, 1, 1, 2, "disabled", True), (1, 1, 1, 2, "every_pipe_stage", True)),
    ((1, 2, 2, 2, "disabled", False), (2, 1, 2, 2, "disabled", False)),
    ((1, 1, 2, 1, "disabled", False), (2, 1, 2, 2, "disabled", False)),
    ((1, 1, 2, 1, "disabled", False), (1, 2, 2, 2, "disabled", False)),
    ((1, 1, 2, 1, "disabled", True), (1, 1, 2, 1, "disabled", False)),
    ((2, 1, 2, 2, "disabled", True), (2, 1, 2, 2, "disabled", False)),
    ((1, 1, 2, 1, "disabled", True), (1, 2, 2, 2, "disabled", True)),
]


@pytest.mark.parametrize("before,after", LAYOUT_CHANGES)
@pytest.mark.parametrize("weight_tying", [False, True])
def test_resume_with_different_layout(tmp_path, before, after, weight_tying):
    """Checkpoint at step 6 under one (TP, PP, DP, ZeRO, checkpointing) layout, resume under another: the
    layout-independent checkpoint must continue the same run (reference tolerance: 15 % on the loss)."""
    _make_data(tmp_path / "data")

    def cfg_for(mp, pp, world, acc, ckpt, zero):
        c = _config(tmp_path, mp, pp, world, checkpointing=ckpt, weight_tying=weight_tying)
        c["topology"]["gradient_accumulation_steps"] = acc
        c["optimizer"]["zero"] = zero
        return c

    full = _run(tmp_path, cfg_for(*before), before[2], "full")
    c2 = cfg_for(*after)
    c2["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, c2, after[2], "resumed")
    for a, b in zip(_losses(full)[-4:], _losses(resumed)):
        assert abs(a - b) / a < 0.15, (_losses(full), _losses(resumed))


def test_activation_checkpointing_does_not_change_losses(tmp_path):
    """Reference test_activation_checkpointing.py: identical losses with and without recomputation."""
    _make_data(tmp_path / "data")
    runs = {}
    for ck in ("disabled", "every_layer", "every_pipe_stage"):
        d = tmp_path / ck
        d.mkdir()
        (d / "data.bin").symlink_to(tmp_path / "data.bin")
        for suffix in (".idx", ".meta.json"):
            (d / f"data{suffix}").symlink_to(tmp_path / f"data{suffix}")
        cfg = _no_dropout(_config(d, 1, 1, 1, checkpointing=ck))
        cfg["trainer"]["save_dir"] = None
        runs[ck] = _losses(_run(d, cfg, 1, "run"))
    np.testing.assert_allclose(runs["every_layer"], runs["disabled"], rtol=1e-6)
    np.testing.assert_allclose(runs["every_pipe_stage"], runs["disabled"], rtol=1e-6)


def test_resume_with_sequence_parallel(tmp_path):
    """Reference test_training_sequence_parallel.py: train without SP, resume with SP (losses within 1e-2)."""
    _make_data(tmp_path / "data")
    cfg = _no_dropout(_config(tmp_path, 2, 1, 2))
    full = _run(tmp_path, cfg, 2, "full")
    c2 = copy.deepcopy(cfg)
    c2["topology"]["sequence_parallel"] = True
    c2["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, c2, 2, "resumed")
    np.testing.assert_allclose(_losses(resumed), _losses(full)[-4:], rtol=1e-2)


@pytest.mark.parametrize("mp,pp,world", [(1, 1, 1), (1, 2, 2), (2, 1, 2)])
def test_load_checkpoint_non_strict(tmp_path, mp, pp, world):
    """Resume into a model with extra softprompt + adapter parameters (allowed missing keys): training continues
    and the new parameters change the losses."""
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, mp, pp, world)
    full = _run(tmp_path, cfg, world, "full")
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    cfg["trainer"]["load_optimizer_states"] = False
    cfg["transformer_architecture"]["softprompt_config"] = {"name": "summarization", "n_tokens": 2}
    cfg["transformer_architecture"]["adapter_config"] = {"name": "image_encoder", "attention_downsampling_factor": 1.0,
                                                         "mlp_downsampling_factor": 1.0}
    cfg["trainer"]["allowed_missing_keys_in_checkpoint"] = [
        "softprompt_summarization", "attn_adapter_image_encoder.dense_in.weight",
        "attn_adapter_image_encoder.dense_out.weight", "mlp_adapter_image_encoder.dense_in.weight",
        "mlp_adapter_image_encoder.dense_out.weight"]
    cfg["training"]["finetune"] = True
    cfg["training"]["finetunable_parameters"] = ["summarization", "image_encoder"]
    resumed = _run(tmp_path, cfg, world, "resumed")
    assert len(resumed) == 4
    for a, b in zip(_losses(full)[-4:], _losses(resumed)):
        assert abs(a - b) > 1e-5


@pytest.mark.parametrize("mp,pp,world", [(1, 1, 1), (2, 1, 2)])
@pytest.mark.parametrize("local_heads", [4, 2])
def test_local_attention_training(tmp_path, mp, pp, world, local_heads):
    """Reference test_training_local_attention.py: sliding-window heads train (finite losses, bit-exact resume);
    local_heads=2 of 4 is the mixed local/global layout (one attention call with a per-head window).  Local
    attention needs the flash kernel path (reference attention.py:319-332)."""
    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, mp, pp, world, masked_softmax={"kernel": "flash_attention"},
                  num_local_attention_heads=local_heads, local_attention_window_size=16)
    full = _run(tmp_path, cfg, world, "full")
    assert all(np.isfinite(_losses(full)))
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, cfg, world, "resumed")
    assert _losses(resumed) == _losses(full)[-4:]


@needs_fixtures
@pytest.mark.parametrize("mp,pp,world", [(1, 1, 1), (1, 2, 2)])
def test_legacy_dataset_training(tmp_path, mp, pp, world):
    """Reference test_training_legacy.py: training on the Megatron MMIDIDX (Enron) fixture, blended x2."""
    cfg = _config(tmp_path, mp, pp, world, vocab_size=128000)
    cfg["data"] = {"data_prefixes": [str(FILES / "dataset" / "legacy" / "enron_text_document_100")] * 2,
                   "legacy_dataset": True, "blended_dataset": {"cache_directory": str(tmp_path)}}
    full = _run(tmp_path, cfg, world, "full")
    assert all(np.isfinite(_losses(full)))
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _run(tmp_path, cfg, world, "resumed")
    assert _losses(resumed) == _losses(full)[-4:]


@needs_fixtures
@pytest.mark.parametrize("mp,pp,world", [(1, 1, 1), (2, 1, 2)])
def test_chat_finetuning_softprompt(tmp_path, mp, pp, world):
    """Reference test_training_finetuning_chat.py: pretrain on chat data, then finetune a softprompt only."""
    tok = FILES / "llama2-tokenizer.json"
    cfg = _config(tmp_path, mp, pp, world, vocab_size=32000, vocab_file=str(tok))
    cfg["data"] = {"data_prefixes": [str(FILES / "dataset" / "finetuning_chat.jsonl")], "finetuning_chat_dataset": True,
                   "blended_dataset": {"cache_directory": str(tmp_path)}}
    _run(tmp_path, cfg, world, "pre")
    cfg["trainer"].update(assert_checkpoint_loaded=True, load_optimizer_states=False, load_context=False,
                          save_interval=2, train_iterations=4, allowed_missing_keys_in_checkpoint=["softprompt_chat"])
    cfg["transformer_architecture"]["softprompt_config"] = {"name": "chat", "n_tokens": 4}
    cfg["training"]["finetune"] = True
    cfg["training"]["finetunable_parameters"] = ["softprompt_chat"]
    ft = _run(tmp_path, cfg, world, "ft")
    assert len(ft) == 4 and all(np.isfinite(_losses(ft)))
    ck = tmp_path / "ckpt"
    s2 = torch.load(str(next((ck / "global_step2").glob("model_state_layer_0_*softprompt*.pt"))), weights_only=True)
    s4 = torch.load(str(next((ck / "global_step4").glob("model_state_layer_0_*softprompt*.pt"))), weights_only=True)
    assert any((s2[k] != s4[k]).any() for k in s2)


# tensors-only fixture of the reference test (copied so the GPU box, which has no reference tree, can run it)
BACKCOMPAT = Path(__file__).resolve().parent / "files" / "backward_compatibility_checkpoint"


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_backward_compatibility_with_legacy_checkpoint(device):
    """Reference test_backwards_compatibility.py: a legacy (pre-`scaling`) 1-layer checkpoint loaded into the
    layer stack reproduces the stored forward activations of every sub-module within 3e-3 (on the GPU: through
    the HIP norm / RoPE / attention / MLP kernels in fp32)."""
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig
    from scaling_amd.transformer.data.text_dataset_batch import TextDatasetBatch
    from scaling_amd.transformer.data.utils import get_cumulative_seq_lengths, get_position_ids
    from scaling_amd.transformer.model.model import get_transformer_layer_specs

    d = BACKCOMPAT
    sd = torch.load(str(d / "state_dict.pt"), weights_only=True)
    gt = torch.load(str(d / "ground_truth.pt"), weights_only=True)
    arch = TransformerArchitectureConfig(vocab_size=512, sequence_length=4, hidden_size=16, num_attention_heads=2,
                                         num_layers=1)
    layers = torch.nn.ModuleList([spec.initialize(device=torch.device(device)) for spec in get_transformer_layer_specs(arch)])

    mapped = {}
    for k, v in sd.items():
        if k.endswith(".inv_freq"):
            continue
        if k == "transformer.embeddings.word_embeddings.weight":
            mapped["0.embedding.weight"] = v
            mapped["3.embedding.weight"] = v
            continue
        if k.startswith("transformer.layer0"):
            k2 = k.replace("transformer.layer0", "1").replace(".attention.", ".self_attention.")
            k2 = k2.replace("dense_h_to_4h", "dense_in").replace("dense_4h_to_h", "dense_out")
        elif k.startswith("transformer.norm"):
            k2 = k.replace("transformer", "2")
        else:
            raise AssertionError(k)
        mapped[k2] = v
    own = layers.state_dict()
    mapped = {k: v for k, v in mapped.items() if k in own}
    missing = set(own) - set(mapped)
    assert not {m for m in missing if not m.endswith(("cos_table", "sin_table"))}, missing
    layers.load_state_dict(mapped, strict=False)
    layers.eval()

    tokens = gt["input"].to(device)
    cu = get_cumulative_seq_lengths(tokens, reset_attention_mask=False)
    pos = get_position_ids(tokens, reset_position_ids=False)
    batch = TextDatasetBatch(input_token_ids=tokens, cumulative_seq_lengths=cu, position_ids=pos)
    with torch.no_grad():
        emb = layers[0](batch)
        out1 = layers[1](emb)
        ln_in = layers[1].input_layernorm(emb.activations)
        attn = layers[1].attention_block(emb.activations, cumulative_seq_lengths=batch.cumulative_seq_lengths,
                                         position_ids=batch.position_ids)
        ln_post = layers[1].post_attention_layernorm(attn)
        mlp = layers[1].mlp_block(attn)
        norm = layers[2](out1)
        logits = layers[3](norm)

    checks = {
        "hidden_states_embedding": emb.activations, "hidden_states_input_layernorm": ln_in,
        "hidden_states_attention": attn, "hidden_states_post_attention_layernorm": ln_post,
        "hidden_states_mlp": mlp, "hidden_states_layer0": out1.hidden(), "hidden_states_norm": norm.activations,
        "output_logits": logits.activations,
    }
    diffs = {k: (gt[k].float() - v.float().cpu()).abs().max().item() for k, v in checks.items()}
    assert all(d < 3e-3 for d in diffs.values()), diffs
