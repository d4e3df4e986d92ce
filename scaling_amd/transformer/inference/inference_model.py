"""Transformer inference (reference ``transformer/inference/inference_model.py``): checkpoint loading
with config + vocab, logits, hidden-state recording and greedy / sampled generation with or
without the KV cache."""
from __future__ import annotations

from pathlib import Path
from typing import Any, Callable, Optional, Sequence

import torch
import yaml

from ...core import BaseLayerIO, LayerSpec, PipePartitionMethod
from ...core.nn.parallel_module.inference_module import InferenceModule, RecorderSetting
from ..context.config import TransformerArchitectureConfig
from ..data import TextDatasetBatch
from ..data.inference_settings import InferenceSettings
from ..model.layers.base import TransformerLayerIO
from ..model.model import get_transformer_layer_specs
from ..tokenizer import Tokenizer
from .sample import sample_argmax


class CompletionOutput:
    def __init__(self, completion_text: Optional[str], completion_tokens: list[int], completion_logits: torch.Tensor):
        self.completion_text = completion_text
        self.completion_tokens = completion_tokens
        self.completion_logits = completion_logits


class TransformerInferenceModule(InferenceModule):
    def __init__(self, layer_specs: list[LayerSpec], devices: Sequence[Any] = (0,),
                 pipe_partition_method: PipePartitionMethod = PipePartitionMethod.UNIFORM,
                 pipe_partition_overwrite: Optional[list[int]] = None, tokenizer: Optional[Tokenizer] = None):
        super().__init__(layer_specs=layer_specs, devices=devices, pipe_partition_method=pipe_partition_method,
                         pipe_partition_overwrite=pipe_partition_overwrite)
        self.tokenizer = tokenizer

    @staticmethod
    def _parse_config_file(config_file: Path) -> TransformerArchitectureConfig:
        with open(config_file, "r") as f:
            d = yaml.safe_load(f)
        return TransformerArchitectureConfig.from_dict(d["transformer_architecture"])

    @classmethod
    def from_checkpoint(cls, checkpoint_dir: Path, devices: Sequence[Any] = (0,),
                        pipe_partition_method: PipePartitionMethod = PipePartitionMethod.UNIFORM,
                        pipe_partition_overwrite: Optional[list[int]] = None, config_file: Optional[Path] = None,
                        vocab_file: Optional[Path] = None) -> "TransformerInferenceModule":
        """Weights, ``config.yml`` and ``vocab.json`` are expected in the checkpoint directory by default."""
        checkpoint_dir = Path(checkpoint_dir)
        config_file = config_file or checkpoint_dir / "config.yml"
        vocab_file = vocab_file or checkpoint_dir / "vocab.json"
        assert config_file.is_file(), "Config file not found"
        assert vocab_file.is_file(), "Vocab file not found"
        arch = cls._parse_config_file(config_file)
        model = cls(layer_specs=get_transformer_layer_specs(architecture_config=arch), devices=devices,
                    pipe_partition_method=pipe_partition_method, pipe_partition_overwrite=pipe_partition_overwrite,
                    tokenizer=Tokenizer.from_file(str(vocab_file)))
        model.load_checkpoint(checkpoint_dir)
        return model

    def forward(self, x: BaseLayerIO) -> TransformerLayerIO:
        out = super().forward(x)
        assert isinstance(out, TransformerLayerIO)
        return out

    def _pre_process_input(self, input_text: Optional[str] = None, input_tokens: Optional[list[int]] = None,
                           process_for_cached_inference: bool = True) -> TextDatasetBatch:
        assert (input_text is None) ^ (input_tokens is None), "Either input_text or input_tokens needs to be provided"
        if input_text is not None:
            assert self.tokenizer is not None
            input_tokens = self.tokenizer.encode(input_text)
        settings = InferenceSettings(use_cache=process_for_cached_inference, reset_cache=True, cache_index=0,
                                     embedding_layers=[-1])
        return TextDatasetBatch(input_token_ids=torch.tensor(input_tokens).unsqueeze(0), inference_settings=settings)

    @staticmethod
    def _post_process_output(output: TransformerLayerIO) -> torch.Tensor:
        return output.activations.squeeze()

    def logits(self, input_text: Optional[str] = None, input_tokens: Optional[list[int]] = None) -> torch.Tensor:
        return self._post_process_output(self.forward(self._pre_process_input(input_text, input_tokens))).squeeze()

    def logits_with_hidden_state_recorder(self, input_text: Optional[str] = None, input_tokens: Optional[list[int]] = None,
                                          recorder_settings_per_layer: Optional[dict[int, RecorderSetting]] = None
                                          ) -> tuple[torch.Tensor, dict[int, dict[str, Any]]]:
        batch = self._pre_process_input(input_text, input_tokens)
        out, rec = super().forward_with_hidden_state_recorder(batch, recorder_settings_per_layer=recorder_settings_per_layer)
        assert isinstance(out, TransformerLayerIO)
        return self._post_process_output(out), rec

    def generate(self, max_tokens: int, input_text: Optional[str] = None, input_tokens: Optional[list[int]] = None,
                 sample_fn: Callable[[torch.Tensor], torch.Tensor] = sample_argmax,
                 stop_tokens: Optional[Sequence[int]] = None, use_cache: bool = True,
                 use_cuda_graph: bool = False) -> CompletionOutput:
        """Completion text / tokens / logits for a prompt.  With the KV cache each step feeds only the new
        token (with its absolute position); without it the whole sequence is re-run.

        ``use_cuda_graph`` (KV cache, one GPU, flash attention, a graph-safe sampler such as ``sample_argmax``):
        after the prefill, the decode step is captured once as a HIP graph and replayed per token
        (``graph_decode.GraphDecoder``) — same kernels and results as the eager loop, without its per-token
        launch and Python overhead."""
        if stop_tokens is None:
            assert self.tokenizer is not None, "If no tokenizer is provided, a stop token needs to be set manually"
            stop_tokens = [self.tokenizer.eos_token_id]
        cur = self._pre_process_input(input_text, input_tokens, process_for_cached_inference=use_cache)
        assert cur.input_token_ids is not None
        n_in = cur.input_token_ids.shape[-1]
        if use_cuda_graph:
            assert use_cache, "graph-captured decoding needs the KV cache"
            return self._generate_graph(cur, n_in, max_tokens, sample_fn, stop_tokens)
        settings = InferenceSettings(use_cache=use_cache, reset_cache=not use_cache, cache_index=0, embedding_layers=[-1])
        tokens: list[int] = []
        step_logits: list[torch.Tensor] = []
        out: Optional[TransformerLayerIO] = None
        for k in range(max_tokens):
            out = self.forward(cur)
            nxt = sample_fn(out.activations)
            tok = int(nxt.item())
            tokens.append(tok)
            if use_cache:
                step_logits.append(out.activations[:, -1, :])
                cur = TextDatasetBatch(input_token_ids=nxt.reshape(1, 1).cpu(), inference_settings=settings,
                                       position_ids=torch.tensor([[n_in + k]]))
            else:
                ids = torch.cat([cur.input_token_ids, nxt.reshape(1, 1).to(cur.input_token_ids.device)], dim=-1)
                cur = TextDatasetBatch(input_token_ids=ids, inference_settings=settings)
            if tok in stop_tokens:
                break
        if use_cache:
            logits = torch.cat(step_logits)
        else:
            assert out is not None
            logits = self._post_process_output(out)[n_in - 1 :]
        text = self.tokenizer.decode(tokens) if self.tokenizer is not None else None
        return CompletionOutput(completion_text=text, completion_tokens=tokens, completion_logits=logits)

    def _generate_graph(self, prompt: TextDatasetBatch, n_in: int, max_tokens: int,
                        sample_fn: Callable[[torch.Tensor], torch.Tensor], stop_tokens: Sequence[int]) -> CompletionOutput:
        from .graph_decode import GraphDecoder

        assert self.devices is not None and len(self.devices) == 1, "graph-captured decoding runs on one device"
        out = self.forward(prompt)  # prefill (reset_cache): fills each layer's KVCache
        first = sample_fn(out.activations)
        assert first.is_cuda, "graph-captured decoding needs a GPU"
        dec = GraphDecoder(self, n_in, max_tokens, first, sample_fn, out.activations[:, -1, :])
        dec.capture()
        tokens, logits = dec.run(stop_tokens)
        text = self.tokenizer.decode(tokens) if self.tokenizer is not None else None
        return CompletionOutput(completion_text=text, completion_tokens=tokens, completion_logits=logits)
