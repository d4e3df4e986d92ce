"""Transformer pipeline model, loss and optimizer wiring (reference ``transformer/model/model.py``).

Differences from the reference that matter for MI355X throughput:

* ``loss_function`` runs the fused HIP cross-entropy over bf16 logits; with tensor parallelism the
  logits stay vocab-sharded (the LM head tags ``TransformerLayerIO.vocab_parallel``) and only per-row
  statistics cross the TP group.  The backward overwrites the logits buffer with the gradient.
* metrics stay on device (no per-micro-batch host sync); one DP all-reduce per step.
* parameter-group bookkeeping uses one all-reduce + one all-gather instead of object collectives.
"""
from __future__ import annotations

import math
import re
from typing import Optional, Sequence, TypeAlias, Union

import torch
import torch.distributed as dist

from ...core import (
    BaseOptimizer,
    CoreParameterMeta,
    LayerSpec,
    Optimizer,
    OptimizerParamGroup,
    OptimizerParamGroupConfig,
    ParallelModule,
    TiedLayerSpec,
    Topology,
)
from ...core.logging import logger
from ...core.nn.parallel_module.buffers import BufferType
from ...ops.xent import vocab_parallel_cross_entropy
from ..context import LearningRateSchedulerConfig, OptimizerConfig, TransformerArchitectureConfig, TransformerContext
from ..context.config import TrainingConfig
from ..data.text_dataset_batch import TextDatasetBatch
from ..data.utils import remove_cumulative_seq_lengths_padding
from .layers import (
    EmbeddingInput,
    LayerNormWrapper,
    TransformerEmbeddingHead,
    TransformerLayer,
    TransformerLayerIO,
    TransformerLMHead,
    TransformerLMHeadTied,
)

NamedParameterMeta: TypeAlias = tuple[str, torch.Tensor, CoreParameterMeta]


def loss_function(output: TransformerLayerIO, batch: TextDatasetBatch) -> tuple[torch.Tensor, dict[str, torch.Tensor]]:
    """Weighted token cross-entropy + accuracy (reference ``model.py:44-77``)."""
    assert batch.target_token_ids is not None, "target_token_ids not set in batch"
    assert batch.loss_weights is not None, "loss_weights not set in batch"
    logits = output.activations
    target = batch.target_token_ids.reshape(-1)
    w = batch.loss_weights.reshape(-1).float()
    if output.vocab_parallel is not None:
        v0, group, tp = output.vocab_parallel
    else:
        v0, group, tp = 0, None, 1
    losses, amax = vocab_parallel_cross_entropy(logits.reshape(-1, logits.shape[-1]), target, v0=v0, group=group, tp=tp,
                                                inplace_grad=torch.is_grad_enabled())
    loss = torch.sum(losses * w) / w.sum()
    mask = (w > 0).float()
    accuracy = torch.sum((amax == target).float() * mask) / mask.sum()
    return loss, {"accuracy": accuracy.detach()}


def metrics_aggregation_fn(topology: Topology, metrics: list[dict[str, torch.Tensor]]) -> dict[str, torch.Tensor]:
    """Mean over micro batches, then over data-parallel ranks (reference ``model.py:80-95``)."""
    out: dict[str, torch.Tensor] = {}
    for k in metrics[0]:
        t = torch.stack([torch.as_tensor(m[k], device=topology.device).float().reshape(()) for m in metrics]).mean()
        if topology.config.data_parallel_size > 1:
            dist.all_reduce(t, group=topology.data_parallel_group)
            t = t / topology.config.data_parallel_size
        out[k] = t
    return out


class TransformerParallelModule(ParallelModule[TransformerLayerIO, TextDatasetBatch]):
    """Drops the un-padded cu_seqlens before pipeline p2p (fixed-shape padded copy travels instead) and
    rebuilds it on receipt (reference ``model.py:98-122``)."""

    def _execute_send_activations(self, buffer_id: int) -> None:
        out = self.pipe_buffer.data[BufferType.PIPELINE_STAGE_OUTPUT][buffer_id]
        assert out is not None
        out.cumulative_seq_lengths = None
        super()._execute_send_activations(buffer_id=buffer_id)

    def _execute_receive_activations(self, buffer_id: int) -> None:
        super()._execute_receive_activations(buffer_id=buffer_id)
        x = self.pipe_buffer.data[BufferType.PIPELINE_STAGE_INPUT][buffer_id]
        assert x is not None
        if x.cumulative_seq_lengths is None:
            assert x.cumulative_seq_lengths_padded is not None
            x.cumulative_seq_lengths = remove_cumulative_seq_lengths_padding(x.cumulative_seq_lengths_padded)


def get_transformer_layer_specs(architecture_config: TransformerArchitectureConfig,
                                topology: Optional[Topology] = None) -> list[LayerSpec]:
    """Embedding → N blocks → final norm → LM head (→ embedding head); small-init std sqrt(2/(5h))
    (reference ``model.py:125-223``)."""
    cfg = architecture_config
    std = math.sqrt(2 / (cfg.hidden_size * 5))

    def init_method(x: torch.Tensor) -> torch.Tensor:
        return torch.nn.init.normal_(x, mean=0.0, std=std)

    specs: list[Union[TiedLayerSpec, LayerSpec]] = []
    tied = ["embedding.weight"] if cfg.weight_tying else []
    common = dict(architecture_config=cfg, topology=topology)
    if cfg.weight_tying:
        specs.append(TiedLayerSpec(module_class=EmbeddingInput, key="embedding_tying", tied_weight_attributes=tied,
                                   init_method=init_method, **common))
    else:
        specs.append(LayerSpec(module_class=EmbeddingInput, init_method=init_method, **common))
    for i in range(cfg.num_layers):
        specs.append(LayerSpec(TransformerLayer, layer_index=i, init_method=init_method, **common))
    specs.append(LayerSpec(LayerNormWrapper, layer_index=cfg.num_layers, **common))
    if cfg.weight_tying:
        specs.append(TiedLayerSpec(module_class=TransformerLMHeadTied, key="embedding_tying", tied_weight_attributes=tied,
                                   init_method=init_method, **common))
    else:
        specs.append(LayerSpec(module_class=TransformerLMHead, init_method=init_method, **common))
    if cfg.embedding_head_config is not None:
        specs.append(LayerSpec(module_class=TransformerEmbeddingHead, **common))
    return specs


def init_model(context: TransformerContext, use_continuous_recommunication: bool = False) -> TransformerParallelModule:
    specs = get_transformer_layer_specs(context.config.transformer_architecture, topology=context.topology)
    return TransformerParallelModule(layer_specs=specs, topology=context.topology, profiler_config=context.config.profiler,
                                     use_continuous_recommunication=use_continuous_recommunication)


def _world() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def get_parameter_groups(context: TransformerContext, model: TransformerParallelModule,
                         learning_rate_scheduler_config: Optional[LearningRateSchedulerConfig] = None,
                         embedding_learning_rate_scheduler_config: Optional[LearningRateSchedulerConfig] = None,
                         ) -> list[OptimizerParamGroup]:
    """Weight-decay / no-decay / separate-lr-embedding groups; groups that are non-empty on ANY rank
    exist on every rank (reference ``model.py:240-324``)."""
    lr_cfg = learning_rate_scheduler_config or context.config.learning_rate_scheduler
    emb_lr_cfg = embedding_learning_rate_scheduler_config or context.config.embedding_learning_rate_scheduler
    emb_wd, no_wd, wd = _extract_parameters(context.config.training, model.named_parameters_with_meta())
    counts = torch.tensor([len(wd), len(no_wd), len(emb_wd)], dtype=torch.long, device=context.topology.device)
    if dist.is_initialized():
        dist.all_reduce(counts, op=dist.ReduceOp.MAX)
    counts_l = counts.tolist()
    assert sum(counts_l) > 0, "did not specify any finetuneable parameters on any rank"
    logger.warning(f"training parameters: {sorted({p[0] for p in wd + no_wd + emb_wd})}")
    groups = []
    training = context.config.training
    if counts_l[0] > 0:
        groups.append(OptimizerParamGroup(wd, OptimizerParamGroupConfig(
            name="weight_decay_params", weight_decay=training.weight_decay, learning_rate_scheduler=lr_cfg)))
    if counts_l[1] > 0:
        groups.append(OptimizerParamGroup(no_wd, OptimizerParamGroupConfig(
            name="no_weight_decay_params", weight_decay=0.0, learning_rate_scheduler=lr_cfg)))
    if counts_l[2] > 0:
        groups.append(OptimizerParamGroup(emb_wd, OptimizerParamGroupConfig(
            name="embedding_weight_decay_params", weight_decay=training.weight_decay, learning_rate_scheduler=emb_lr_cfg)))
    assert groups, "Number of optimizer groups is zero"
    return groups


def _extract_parameters(training_config: TrainingConfig, named_parameters_with_meta: list[NamedParameterMeta],
                        ) -> tuple[list[NamedParameterMeta], list[NamedParameterMeta], list[NamedParameterMeta]]:
    wd: list[NamedParameterMeta] = []
    no_wd: list[NamedParameterMeta] = []
    emb: list[NamedParameterMeta] = []
    found: set[str] = set()
    for npm in named_parameters_with_meta:
        if training_config.finetune:
            match = _find_matching_param(npm, training_config.finetunable_parameters)
            if match is None:
                continue
            found.add(match)
        name = npm[0]
        if name.endswith(".bias"):
            no_wd.append(npm)
        elif training_config.use_separate_lr_on_embeddings and name == "embedding.weight":
            assert not training_config.finetune, "Can not use separate lr on embeddings with finetuning"
            emb.append(npm)
        else:
            wd.append(npm)
    unmatched = _find_global_unmatched_parameters(found, training_config.finetunable_parameters)
    if unmatched:
        raise ValueError(f"Unmatched finetunable parameters: {unmatched}")
    if training_config.parameters_exclude:
        ex = training_config.parameters_exclude
        wd, no_wd, emb = (_filter_by_param(ex, lst) for lst in (wd, no_wd, emb))
    return emb, no_wd, wd


def _find_global_unmatched_parameters(found: set[str], finetunable_parameters: Sequence[str]) -> set[str]:
    """Patterns matched on no rank at all.  Encoded as a 0/1 vector and MIN-reduced over the world."""
    pats = list(finetunable_parameters)
    if not pats:
        return set()
    miss = torch.tensor([0 if p in found else 1 for p in pats], dtype=torch.int32)
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            miss = miss.cuda()
        dist.all_reduce(miss, op=dist.ReduceOp.MIN)
    return {p for p, m in zip(pats, miss.tolist()) if m}


def _filter_by_param(parameters_exclude: list[str], parameter_list: list[NamedParameterMeta]) -> list[NamedParameterMeta]:
    return [p for p in parameter_list if _find_matching_param(p, parameters_exclude) is None]


def _find_matching_param(key: NamedParameterMeta, data: Sequence[str]) -> Optional[str]:
    return next((item for item in data if re.search(item, key[0]) is not None), None)


def init_optimizer(context: TransformerContext, model: TransformerParallelModule,
                   optimizer_config: Optional[OptimizerConfig] = None,
                   learning_rate_scheduler_config: Optional[LearningRateSchedulerConfig] = None,
                   embedding_learning_rate_scheduler_config: Optional[LearningRateSchedulerConfig] = None) -> BaseOptimizer:
    groups = get_parameter_groups(context, model, learning_rate_scheduler_config, embedding_learning_rate_scheduler_config)
    # parameters outside every group are frozen: autograd skips their weight gradients entirely
    trained = {id(p) for g in groups for p in g.parameters_original}
    for _, p, _ in model.named_parameters_with_meta():
        if id(p) not in trained:
            p.requires_grad_(False)
    return Optimizer(config=optimizer_config or context.config.optimizer, parameter_groups=groups, topology=context.topology)
