"""Pre-norm transformer block (reference ``model/layers/layer.py:44-291``): attention block and MLP
block with residuals, dropouts under the TP-constant RNG, optional bottleneck adapters."""
from __future__ import annotations

import os
from functools import partial
from typing import Callable, Optional, Union

import torch

from ....core import ParallelMLP, ParallelSelfAttention, ParallelSwiGLUMLP, RotaryConfig, Topology, get_norm
from ....core.utils.grad_probe import probe
from ....ops.attention import stash_active
from ....ops.elementwise import dropout_add
from ...context.config import MLPType, TransformerArchitectureConfig
from .base import TransformerLayerBaseIO, TransformerLayerIO
from .embedding import _device

# decode-sized MLP blocks on the fused GEMV epilogues (SwiGLU, residual add); SCALING_AMD_DECODE_FUSED=0 for A/B
_DECODE_FUSED = os.environ.get("SCALING_AMD_DECODE_FUSED", "1") != "0"
# decode-sized RMSNorms as prologues of the following GEMVs; SCALING_AMD_DECODE_NORM_GEMV=0 for A/B
_DECODE_NORM_GEMV = _DECODE_FUSED and os.environ.get("SCALING_AMD_DECODE_NORM_GEMV", "1") != "0"
# hand the MLP's residual add to the next layer's add-norm kernel (TransformerLayerIO.residual_branch);
# SCALING_AMD_DEFER_RESIDUAL=0 for A/B
_DEFER_RESIDUAL = os.environ.get("SCALING_AMD_DEFER_RESIDUAL", "1") != "0"
# sequence parallelism: the norms hand their token shard to the q/k/v and gate/up GEMMs, which gather it overlapped
# with the GEMM (core/nn/linear/tp_overlap.py: sp_gather_column); SCALING_AMD_SP_OVERLAP=0 gathers in the norms
_SP_OVERLAP = os.environ.get("SCALING_AMD_SP_OVERLAP", "1") != "0"


def residual_defer_allowed(topology: Optional[Topology]) -> bool:
    """Whether a layer may leave its MLP residual add pending under this topology's checkpointing: not when every
    layer's input is a checkpoint boundary (every_layer*: the pending pair would be saved as two tensors)."""
    ac = getattr(getattr(topology, "config", None), "activation_checkpointing_type", None)
    return _DEFER_RESIDUAL and "every_layer" not in str(getattr(ac, "value", ac))


class ZeroLayer(torch.nn.Module):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.zeros_like(x)


def get_batched_adapter_forward(adapter_list: list[Optional[torch.nn.Module]]) -> Callable[[torch.Tensor], torch.Tensor]:
    mods = [a if a is not None else ZeroLayer() for a in adapter_list]

    def forward(x: torch.Tensor) -> torch.Tensor:
        assert x.shape[0] == len(mods)
        return torch.stack([m(x[i]) for i, m in enumerate(mods)], dim=0)

    return forward


class TransformerLayer(TransformerLayerBaseIO):
    def __init__(self, architecture_config: TransformerArchitectureConfig, layer_index: int,
                 topology: Optional[Topology] = None,
                 init_method: Callable[[torch.Tensor], torch.Tensor] = torch.nn.init.xavier_normal_) -> None:
        super().__init__()
        cfg = architecture_config
        self.architecture_config = cfg
        self.topology = topology
        self.layer_index = layer_index
        # whether this layer may hand its MLP residual add to the next layer (residual_branch): not across a pipeline
        # stage boundary (set_stage_output) and not when every layer's input is a checkpoint boundary (the pending
        # pair would be saved as two tensors instead of one)
        self._defer_ok = residual_defer_allowed(topology)
        dev = _device(topology)
        bitfit = getattr(cfg.bitfit_bias_config, "name", None)
        dtype = cfg.precision.dtype
        self.input_layernorm = get_norm(cfg.norm_type, cfg.layernorm, cfg.hidden_size, dev, dtype, bitfit, topology)
        head_dim = cfg.hidden_size // cfg.num_attention_heads
        self.self_attention = ParallelSelfAttention(
            hidden_size=cfg.hidden_size, num_attention_heads=cfg.num_attention_heads,
            num_local_attention_heads=cfg.num_local_attention_heads,
            local_attention_window_size=cfg.local_attention_window_size, masked_softmax_config=cfg.masked_softmax,
            causal=cfg.causal, dropout_attention_probs=cfg.dropout_attention_probs,
            rotary_config=RotaryConfig(dimensions=int(cfg.rotary_percentage * head_dim), max_seq_length=cfg.sequence_length,
                                       base=cfg.rotary_embedding_base),
            relative_position_embedding_type=cfg.relative_position_embedding_type, bias=cfg.attention_bias,
            topology=topology, device=None if topology is not None else dev, dtype=dtype, bitfit_bias_name=bitfit,
            init_method=init_method, lora_config=cfg.lora_config, norm_type=cfg.norm_type, key_query_norm=cfg.key_query_norm,
            layernorm_config=cfg.layernorm, qkv_in_one=cfg.attention_qkv_in_one, num_kv_heads=cfg.attention_num_kv_heads,
            use_matmul=cfg.attention_use_matmul,
        )
        self.dropout_attention = torch.nn.Dropout(cfg.dropout_after_attention)
        self.post_attention_layernorm = get_norm(cfg.norm_type, cfg.layernorm, cfg.hidden_size, dev, dtype, bitfit, topology)
        mlp_kw = dict(io_features=cfg.hidden_size, intermediate_feature_factor=cfg.mlp_factor, bias=cfg.mlp_bias,
                      topology=topology, device=None if topology is not None else dev, dtype=dtype,
                      bitfit_bias_name=bitfit, init_method=init_method)
        self.mlp: Union[ParallelMLP, ParallelSwiGLUMLP]
        if cfg.mlp_type == MLPType.DEFAULT:
            self.mlp = ParallelMLP(**mlp_kw)
        elif cfg.mlp_type == MLPType.SWIGLU:
            self.mlp = ParallelSwiGLUMLP(**mlp_kw)
        else:
            raise NotImplementedError(str(cfg.mlp_type))
        self.dropout_mlp = torch.nn.Dropout(cfg.dropout_after_mlp)
        if cfg.adapter_config is not None:
            self.load_adapter()

    def load_adapter(self) -> None:
        ac = self.architecture_config.adapter_config
        assert ac is not None
        dev = _device(self.topology)
        kw = dict(io_features=self.architecture_config.hidden_size, bias=False, topology=self.topology,
                  device=None if self.topology is not None else dev, dtype=self.architecture_config.precision.dtype,
                  init_method=partial(torch.nn.init.normal_, mean=0.0, std=ac.init_std))
        if ac.attention_downsampling_factor is not None:
            self.attn_adapter_name = f"attn_adapter_{ac.name}"
            setattr(self, self.attn_adapter_name, ParallelMLP(intermediate_feature_factor=ac.attention_downsampling_factor, **kw))
        if ac.mlp_downsampling_factor is not None:
            self.mlp_adapter_name = f"mlp_adapter_{ac.name}"
            setattr(self, self.mlp_adapter_name, ParallelMLP(intermediate_feature_factor=ac.mlp_downsampling_factor, **kw))

    def apply_adapter(self, x: torch.Tensor, adapter_name: str) -> torch.Tensor:
        assert hasattr(self, adapter_name), f"cannot use adapter '{adapter_name}' as it is not initialized"
        return getattr(self, adapter_name)(x)

    def _dropout_add(self, drop: torch.nn.Dropout, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
        """residual + dropout(x): one fused HIP pass on GPU, under the TP-constant RNG stream."""
        if drop.p == 0.0 or not self.training:
            return residual + x
        if self.topology is not None:
            with self.topology.model_parallel_constant_rng():
                return dropout_add(x, residual, drop.p, True)
        return dropout_add(x, residual, drop.p, True)

    def _attention_delta(self, hidden_state: torch.Tensor, cumulative_seq_lengths: torch.Tensor,
                         position_ids: torch.Tensor, use_cache: bool, reset_cache: bool, cache_index: int,
                         attention_scores_manipulation: Optional[torch.Tensor],
                         attentions_score_manipulation_log_additive: Union[bool, list[bool]]) -> torch.Tensor:
        h = self.input_layernorm(hidden_state)
        return self.self_attention(
            h, cumulative_seq_lengths=cumulative_seq_lengths, position_ids=position_ids, use_cache=use_cache,
            reset_cache=reset_cache, cache_index=cache_index, attention_scores_manipulation=attention_scores_manipulation,
            attentions_score_manipulation_log_additive=attentions_score_manipulation_log_additive,
        )

    def _sp_overlap(self, decode_step: bool) -> bool:
        """Whether this forward hands sequence-parallel norm shards to their GEMMs (``_SP_OVERLAP``): TP > 1 with
        sequence parallelism, a training-shaped step, attention without unmerged LoRA, outside a GEMM-keeping
        checkpoint region (whose replay would re-run the gather)."""
        if not _SP_OVERLAP or decode_step or self.topology is None or stash_active():
            return False
        return self.self_attention.sp_shard_eligible()

    def _mlp_tail(self, residual: torch.Tensor, normed: torch.Tensor, sp_shard: bool = False) -> torch.Tensor:
        out = None
        fused = getattr(self.mlp, "decode_forward_residual", None) if _DECODE_FUSED and not sp_shard else None
        if fused is not None and (self.dropout_mlp.p == 0.0 or not self.training):
            out = fused(normed, residual)  # decode-sized rows: GEMV epilogues (SwiGLU, residual add)
        if out is None:
            mlp_out = self.mlp(normed, sp_shard=True) if sp_shard else self.mlp(normed)
            out = self._dropout_add(self.dropout_mlp, mlp_out, residual)
        if hasattr(self, "mlp_adapter_name"):
            out = out + self.apply_adapter(out, self.mlp_adapter_name)
        return out

    def attention_block(self, hidden_state: torch.Tensor, cumulative_seq_lengths: torch.Tensor, position_ids: torch.Tensor,
                        use_cache: bool = False, reset_cache: bool = False, cache_index: int = 0,
                        attention_scores_manipulation: Optional[torch.Tensor] = None,
                        attentions_score_manipulation_log_additive: Union[bool, list[bool]] = True) -> torch.Tensor:
        h = self._attention_delta(hidden_state, cumulative_seq_lengths, position_ids, use_cache, reset_cache, cache_index,
                                  attention_scores_manipulation, attentions_score_manipulation_log_additive)
        out = self._dropout_add(self.dropout_attention, h, hidden_state)
        if hasattr(self, "attn_adapter_name"):
            out = out + self.apply_adapter(out, self.attn_adapter_name)
        return out

    def mlp_block(self, hidden_state: torch.Tensor) -> torch.Tensor:
        return self._mlp_tail(hidden_state, self.post_attention_layernorm(hidden_state))

    def set_stage_output(self, last_of_stage: bool) -> None:
        """Called by the pipeline partitioner on the last layer of a stage that sends its output to the next stage."""
        if last_of_stage:
            self._defer_ok = False

    def forward(self, x: TransformerLayerIO) -> TransformerLayerIO:
        st = x.inference_settings
        assert x.cumulative_seq_lengths is not None
        pending = probe(f"layer{self.layer_index}.branch_in", x.residual_branch)  # the previous layer's MLP output,
        probe(f"layer{self.layer_index}.input", x.activations)                # its residual add not done yet
        decode_step = _DECODE_NORM_GEMV and st is not None and st.use_cache and not st.reset_cache
        fused_path = (self.dropout_attention.p == 0.0 or not self.training) and not hasattr(self, "attn_adapter_name")
        hidden = x.activations if (pending is None or (fused_path and not decode_step)) else x.hidden()
        attn_args = (hidden, x.cumulative_seq_lengths, x.position_ids,
                     st.use_cache if st else False, st.reset_cache if st else False, st.cache_index if st else 0,
                     x.attention_scores_manipulation, st.control_log_additive_batch if st else True)
        capture = st is not None and (self.layer_index + 1) in st.embedding_layers
        if fused_path:
            # residual stream through the fused norms: input_layernorm adds the previous layer's pending MLP output
            # (or, without one, folds the residual-branch gradient into its backward); post_attention_layernorm writes
            # x + attn and norm(x + attn) in one pass
            # (decode-sized rows: both norms run as prologues of the q/k/v and gate/up GEMVs instead)
            # only on real decode steps (a cached step after the prompt): the fold keeps the normalised row in fp32, so
            # a short prompt, eval or scoring batch must take the same norm + GEMM path as any longer input
            proj = getattr(self.self_attention, "decode_norm_project", None) if decode_step else None
            kw = proj(hidden, self.input_layernorm, attn_args[2], attn_args[3], attn_args[4],
                      attn_args[5]) if proj is not None else None
            sp = kw is None and self._sp_overlap(decode_step)
            if kw is None:
                kw = {}
                resid, normed = self.input_layernorm.forward_add(hidden, pending if hidden is x.activations else None,
                                                                 gather=not sp)
                if sp:  # normed is this rank's token shard: the q/k/v GEMM gathers it, overlapped
                    kw = {"projected_base": self.self_attention.project_sp_shard(normed)}
            else:
                resid = normed = hidden
            h = self.self_attention(
                normed, cumulative_seq_lengths=attn_args[1], position_ids=attn_args[2], use_cache=attn_args[3],
                reset_cache=attn_args[4], cache_index=attn_args[5], attention_scores_manipulation=attn_args[6],
                attentions_score_manipulation_log_additive=attn_args[7], **kw)
            act = None
            if (decode_step and (self.dropout_mlp.p == 0.0 or not self.training)
                    and not hasattr(self, "mlp_adapter_name")):
                fused = getattr(self.mlp, "decode_forward_norm", None)
                act = fused(h, resid, self.post_attention_layernorm) if fused is not None else None
            if act is None:
                resid, normed = self.post_attention_layernorm.forward_add(resid, h, gather=not sp)
                if (self._defer_ok and not decode_step and not capture and not hasattr(self, "mlp_adapter_name")
                        and (self.dropout_mlp.p == 0.0 or not self.training)):
                    # leave resid + mlp(normed) to the next layer's add-norm (or the final norm)
                    branch = self.mlp(normed, sp_shard=True) if sp else self.mlp(normed)
                    return x.derive(resid, embeddings_head=None, residual_branch=branch)
                act = self._mlp_tail(resid, normed, sp_shard=sp)
        else:
            act = self.mlp_block(self.attention_block(*attn_args))
        if capture:
            assert x.embeddings is not None
            x.embeddings[st.embedding_layers.index(self.layer_index + 1)] = act
        return x.derive(act, embeddings_head=None)
