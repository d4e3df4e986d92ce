"""Input embedding layer (reference ``model/layers/embedding.py:29-375``): vocab-parallel embedding
(HIP gather kernel), dropout under the TP-constant RNG, optional image embeddings, softprompt, and
AtMan-style attention-score manipulation for inference."""
from __future__ import annotations

import collections
from typing import Any, Callable, Optional, TypeVar

import torch

from ....core import BaseLayer, Topology, VocabParallelEmbedding
from ....ops.elementwise import dropout_add
from ...context.config import TransformerArchitectureConfig
from ...data.text_dataset_batch import TextDatasetBatch
from .base import TransformerLayerIO

TextDatasetBatchGeneric = TypeVar("TextDatasetBatchGeneric", bound=TextDatasetBatch)


def _device(topology: Optional[Topology]) -> torch.device:
    if topology is not None:
        return topology.device
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class BaseEmbeddingInput(BaseLayer[TextDatasetBatchGeneric, TransformerLayerIO, TransformerLayerIO]):
    def __init__(self, architecture_config: TransformerArchitectureConfig, topology: Optional[Topology] = None,
                 init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_):
        super().__init__()
        cfg = architecture_config
        self.architecture_config = cfg
        self.topology = topology
        dev = _device(topology)
        self.embedding = VocabParallelEmbedding(
            num_embeddings=cfg.vocab_size, embedding_dim=cfg.hidden_size, topology=topology,
            dtype=cfg.precision.dtype, init_method=init_method, finetunable_token_ids=cfg.finetunable_token_ids,
            device=None if topology is not None else dev,
        )
        self.dropout = torch.nn.Dropout(p=cfg.dropout_embedding)
        if cfg.image_encoder:
            from ..image_encoder import ImageEncoder

            self.image_encoder = ImageEncoder(out_features=cfg.hidden_size, dropout_p=cfg.dropout_image_encoder,
                                              layernorm_config=cfg.layernorm, dtype=cfg.precision.dtype, device=dev)
        self.softprompt_name: Optional[str] = None
        if cfg.softprompt_config is not None:
            self.softprompt_name = cfg.softprompt_config.name
            sp = torch.nn.Parameter(torch.zeros(cfg.softprompt_config.n_tokens, cfg.hidden_size,
                                                dtype=cfg.precision.dtype, device=dev))
            init_method(sp)
            setattr(self, f"softprompt_{self.softprompt_name}", sp)
        self.cache: dict[int, Optional[torch.Tensor]] = {}

    def _tp_dropout(self, x: torch.Tensor) -> torch.Tensor:
        if self.dropout.p == 0.0 or not self.training:
            return x
        if self.topology is not None:
            with self.topology.model_parallel_constant_rng():
                return dropout_add(x, None, self.dropout.p, True)
        return dropout_add(x, None, self.dropout.p, True)

    def forward(self, x: TextDatasetBatchGeneric) -> TransformerLayerIO:
        st = x.inference_settings
        use_cache = st.use_cache if st is not None else False
        reset_cache = st.reset_cache if st is not None else False
        cache_index = st.cache_index if st is not None else 0
        if reset_cache:
            self.cache[cache_index] = None
        assert x.input_token_ids is not None
        act = self._tp_dropout(self.embedding(x.input_token_ids))
        if x.input_images is not None:
            if self.topology is not None:
                with self.topology.model_parallel_constant_rng():
                    img = self.image_encoder(x.input_images)
            else:
                img = self.image_encoder(x.input_images)
            locs = x.input_image_locations if x.input_image_locations is not None else (st.input_image_locations if st is not None else None)
            if locs is not None:
                act = act.clone()
                for emb, (bi, s0, s1) in zip(img, locs):
                    act[int(bi), int(s0) : int(s1)] = emb
            else:
                act = torch.cat([img, act[:, img.shape[1] :, :]], dim=1).contiguous()
        if self.softprompt_name is not None:
            sp = getattr(self, f"softprompt_{self.softprompt_name}")
            act = torch.cat([sp.unsqueeze(0).expand(act.shape[0], -1, -1), act[:, sp.shape[0] :, :]], dim=1).contiguous()
        if st is not None and 0 in st.embedding_layers:
            assert x.embeddings is not None
            x.embeddings[0] = act
        loss_weights = x.loss_weights
        manip = None
        if st is not None and st.inference_control_parameters is not None:
            manip = self._attention_manipulation(act, x, use_cache, reset_cache, cache_index)
        out = TransformerLayerIO(
            activations=act, position_ids=x.position_ids, cumulative_seq_lengths=x.cumulative_seq_lengths,
            cumulative_seq_lengths_padded=x.cumulative_seq_lengths_padded, attention_scores_manipulation=manip,
            loss_weights=loss_weights, inference_settings=st, embeddings=x.embeddings,
        )
        return out

    # ------------------------------------------------------------------ AtMan controls
    def _attention_manipulation(self, act: torch.Tensor, x: Any, use_cache: bool, reset_cache: bool, cache_index: int) -> torch.Tensor:
        st = x.inference_settings
        params = st.inference_control_parameters
        b, s = act.shape[0], act.shape[1]
        assert len(params) == b, "number of inference_control_parameters does not match batch size"
        manip = torch.zeros(b, 1, s, s, device=act.device, dtype=act.dtype)
        for i, p in enumerate(params):
            if not p.control_log_additive:
                manip[i] = 1.0
        sim = None
        if any(p.contextual_control_threshold is not None for p in params):
            a = act
            if use_cache:
                if not reset_cache:
                    prev = self.cache[cache_index]
                    assert prev is not None
                    a = torch.cat([prev, a], dim=1)
                self.cache[cache_index] = a
            sim = self.get_embedding_similarity_matrix(a)
        for i, p in enumerate(params):
            if p is None or p.controls is None or all(c.token_index == -1 for c in p.controls):
                continue
            factors: dict[int, float] = collections.defaultdict(lambda: 0.0)
            for c in p.controls:
                if c.token_index < 0:
                    continue
                factors[c.token_index] = c.factor
                if p.contextual_control_threshold is not None:
                    assert sim is not None
                    scores = sim[i][c.token_index]
                    for j in (scores >= p.contextual_control_threshold).nonzero().view(-1).tolist():
                        if j == c.token_index:
                            continue
                        f = self.get_control_factor_from_cosine_similarity(c.factor, scores[j].item())
                        factors[j] = min(f, factors[j])
            for j, f in factors.items():
                if reset_cache:
                    assert x.loss_weights is not None
                    x.loss_weights[i, j] = x.loss_weights[i, j] * f
                if p.control_log_additive:
                    manip[i, :, :, j] = -10000.0 if f == 0.0 else float(torch.log(torch.tensor(f)))
                else:
                    manip[i, :, :, j] = f
        return manip

    def get_control_factor_from_cosine_similarity(self, control_factor: float, cosine_similarity: float) -> float:
        if 0 <= cosine_similarity <= 1.0:
            return (1 - control_factor) * (1 - cosine_similarity) + control_factor
        return 1.0

    def get_embedding_similarity_matrix(self, embeddings: torch.Tensor) -> torch.Tensor:
        assert embeddings.ndim == 3
        with torch.no_grad():
            e = embeddings.float()
            n = e.norm(dim=-1, keepdim=True).clamp_min(1e-8)
            en = e / n
            return torch.bmm(en, en.transpose(1, 2)).cpu().clip(-1, 1)

    def get_similarity_matrix(self, a: torch.Tensor, b: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
        an = a / a.norm(dim=1, keepdim=True).clamp_min(eps)
        bn = b / b.norm(dim=1, keepdim=True).clamp_min(eps)
        return an @ bn.t()

    @staticmethod
    def input_to_tuple(input: Any) -> tuple[Any, ...]:
        return input.as_tuple()

    @staticmethod
    def tuple_to_input(d: tuple[Any, ...]) -> Any:
        return TextDatasetBatch.from_tuple(d)

    @staticmethod
    def output_to_tuple(output: TransformerLayerIO) -> tuple[Any, ...]:
        return output.as_tuple()

    @staticmethod
    def tuple_to_last_stage_activation(d: tuple[Any, ...]) -> TransformerLayerIO:
        return TransformerLayerIO.from_tuple(d)


class EmbeddingInput(BaseEmbeddingInput[TextDatasetBatch]):
    pass
