"""Checkpoint-driven inference (reference tests/transformer/test_inference.py:48-176).

A tiny Llama-style model is trained for a few steps through the training entry point, which saves the weights,
``config.yml`` and ``vocab.json`` with the checkpoint (as ``transformer/train.py`` does).  The run is reloaded with
``TransformerInferenceModule.from_checkpoint`` and checked:

* ``logits`` equal the training-side forward of the same checkpoint (``TransformerParallelModule.load_checkpoint``);
* tokenizer-driven ``generate`` with the KV cache equals ``generate`` without it (tokens and logits);
* the cached decode logits track a full no-cache forward of prompt + completion (pins the decode path's tolerance:
  exact up to fp32 reassociation on CPU, bf16 tolerance on the GPU twin, where decode steps run the fused GEMV
  kernels);
* sampled generation (top-k / top-p / temperature) and the hidden-state recorder scenarios run.

The vocabulary is a byte-level BPE trained in the test with HF ``tokenizers`` (no tokenizer file ships with the
repository); the GPU twin repeats the checks on ``cuda:0`` in bf16.
"""
from __future__ import annotations

from pathlib import Path

import pytest
import torch

from tests.test_training import _config, _make_data, _run

CORPUS = ["the quick brown fox jumps over the lazy dog", "a stitch in time saves nine",
          "all that glitters is not gold", "the early bird catches the worm", "actions speak louder than words",
          "better late than never", "birds of a feather flock together", "the pen is mightier than the sword"]
PROMPT = "the quick brown fox"


def _tokenizer(path: Path) -> None:
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=320, special_tokens=["<|endoftext|>"], show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(CORPUS * 20, tr)
    tok.save(str(path))


def _train_run(tmp: Path, precision: str = "float32") -> tuple[Path, Path]:
    """Trains 4 steps and saves global_step4 (+ vocab.json next to it); returns (checkpoint dir, vocab file)."""
    _make_data(tmp / "data")
    _tokenizer(tmp / "tok.json")
    cfg = _config(tmp, 1, 1, 1, vocab_file=str(tmp / "tok.json"), precision=precision)
    cfg["trainer"].update(train_iterations=4, save_interval=4)
    cfg.pop("profiler", None)
    metrics = _run(tmp, cfg, 1, "train")
    assert len(metrics) == 4
    return tmp / "ckpt" / "global_step4", tmp / "ckpt" / "vocab.json"


def _training_side_logits(ckpt: Path, tokens: list[int], device: str) -> torch.Tensor:
    from scaling_amd.core import Topology, TopologyConfig
    from scaling_amd.transformer.context.config import TransformerConfig
    from scaling_amd.transformer.data.text_dataset_batch import TextDatasetBatch
    from scaling_amd.transformer.model.model import TransformerParallelModule, get_transformer_layer_specs

    cfg = TransformerConfig.from_yaml(ckpt / "config.yml")
    topo = Topology(TopologyConfig(global_rank=0, world_size=1, local_slot=0, model_parallel_size=1,
                                   pipe_parallel_size=1, data_parallel_size=1, micro_batch_size=1,
                                   gradient_accumulation_steps=1, backend="gloo" if device == "cpu" else None))
    topo.initialize_device()
    pm = TransformerParallelModule(get_transformer_layer_specs(cfg.transformer_architecture, topology=topo),
                                   topology=topo)
    pm.load_checkpoint(ckpt)
    pm.eval()
    batch = TextDatasetBatch(input_token_ids=torch.tensor([tokens]))
    batch.to_(topo.device)
    with torch.no_grad():
        return pm(batch).activations[0].float().cpu()


def _check(tmp: Path, device, precision: str, atol: float) -> None:
    from scaling_amd.core.nn.parallel_module.inference_module import RecorderSetting
    from scaling_amd.transformer.inference import (TransformerInferenceModule, sample_temperature, top_k_transform,
                                                   top_p_transform)
    from scaling_amd.transformer.model.layers.base import TransformerLayerIO

    ckpt, vocab = _train_run(tmp, precision)
    assert (ckpt / "config.yml").is_file() and vocab.is_file()
    m = TransformerInferenceModule.from_checkpoint(ckpt, vocab_file=vocab, devices=(device,))
    assert m.tokenizer is not None
    tokens = m.tokenizer.encode(PROMPT)
    assert len(tokens) >= 3

    # logits == the training-side forward of the same weights
    logits = m.logits(input_text=PROMPT).float().cpu()
    assert logits.shape == (len(tokens), 1024)
    ref = _training_side_logits(ckpt, tokens, "cpu" if device == "cpu" else "cuda")
    torch.testing.assert_close(logits, ref, rtol=0, atol=atol / 10 if device == "cpu" else atol)

    # tokenizer-driven generation: cached == uncached
    eos = m.tokenizer.eos_token_id
    a = m.generate(max_tokens=8, input_text=PROMPT, stop_tokens=[eos], use_cache=True)
    b = m.generate(max_tokens=8, input_text=PROMPT, stop_tokens=[eos], use_cache=False)
    assert a.completion_text is not None and b.completion_text is not None
    assert a.completion_tokens == b.completion_tokens
    torch.testing.assert_close(a.completion_logits.float(), b.completion_logits.float(), rtol=0, atol=atol)
    assert a.completion_text == m.tokenizer.decode(a.completion_tokens)

    # cached decode logits vs ONE full no-cache forward of prompt + completion (the decode path's tolerance)
    full = m.logits(input_tokens=tokens + a.completion_tokens).float().cpu()
    n = len(a.completion_tokens)
    torch.testing.assert_close(a.completion_logits.float().cpu(), full[len(tokens) - 1 : len(tokens) - 1 + n],
                               rtol=0, atol=atol)

    # sampled generation
    torch.manual_seed(0)
    s = m.generate(max_tokens=8, input_text=PROMPT, stop_tokens=[eos],
                   sample_fn=lambda x: sample_temperature(top_p_transform(top_k_transform(x))))
    assert 1 <= len(s.completion_tokens) <= 8

    # hidden-state recorder: every layer / the last transformer layer / the attention sub-modules
    n_layers = len(m._layers)
    lg, rec = m.logits_with_hidden_state_recorder(input_text=PROMPT, recorder_settings_per_layer={
        k: RecorderSetting() for k in range(n_layers)})
    assert set(rec) == set(range(n_layers))
    assert all(set(v) == {""} and isinstance(v[""], TransformerLayerIO) for v in rec.values())
    _, rec = m.logits_with_hidden_state_recorder(input_text=PROMPT, recorder_settings_per_layer={
        1: RecorderSetting(include_modules=("self_attention",)), 2: RecorderSetting(include_modules=("self_attention",))})
    assert set(rec) == {1, 2}
    assert all(set(v) == {"self_attention"} and isinstance(v["self_attention"], torch.Tensor) for v in rec.values())
    torch.testing.assert_close(lg.float().cpu(), logits)


@pytest.mark.cpu
def test_inference_from_training_checkpoint_cpu(tmp_path):
    _check(tmp_path, "cpu", "float32", atol=1e-4)


@pytest.mark.gpu
def test_inference_from_training_checkpoint_gpu(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _check(tmp_path, 0, "bfloat16", atol=6e-2)
