"""Throughput accounting (reference ``transformer/utils/get_tflops.py``): the four TFLOP/s estimates
and PaLM MFU, plus tokens/s.  ``HardwareType`` knows the MI355X dense peak (bf16 2.5 PF; no sparsity)."""
from __future__ import annotations

from enum import Enum
from typing import Any

import torch

from ...core.logging import logger
from ...core.topology.topology_config import ActivationCheckpointingType
from ..context.config import TransformerArchitectureConfig

_GELU, _SOFTMAX, _DROPOUT, _NORM = 8, 5, 4, 5


def _layer_flops_per_token(a: TransformerArchitectureConfig, rotary_flops: int) -> int:
    """Electra-style op count of one transformer layer per token (GELU MLP with factor 4 as in the reference)."""
    h, s, n = a.hidden_size, a.sequence_length, a.num_attention_heads
    attention = (_NORM + 6 * h * h + 3 * h + 2 * h * s + _SOFTMAX * s * n + rotary_flops * h + _DROPOUT * s * n + s * n
                 + 2 * s * h + 2 * h * h + h + _DROPOUT * h + h)
    mlp = _NORM + 8 * h * h + 4 * h + _GELU * 4 * h + 8 * h * h + h + _DROPOUT * h + h
    return attention + mlp


def _electra_like(iter_time_s: float, topology: Any, a: TransformerArchitectureConfig, rotary_flops: int,
                  embedding: bool, backward_multiplier: int) -> float:
    tokens = topology.config.global_batch_size * a.sequence_length
    layers = a.num_layers * tokens * _layer_flops_per_token(a, rotary_flops)
    head = 2 * tokens * a.hidden_size * a.vocab_size
    emb = head if embedding else 0
    assert topology.config.world_size is not None
    return backward_multiplier * (emb + layers + _NORM + head) / (iter_time_s * topology.config.world_size * 1e12)


def get_tflops_aleph_alpha(iter_time_s: float, topology: Any, transformer_architecture: TransformerArchitectureConfig) -> float:
    """Electra count with rotary (6 ops/elem), no embedding flops, backward = 2x forward."""
    return _electra_like(iter_time_s, topology, transformer_architecture, 6, False, 3)


def get_tflops_electra(iter_time_s: float, topology: Any, transformer_architecture: TransformerArchitectureConfig) -> float:
    return _electra_like(iter_time_s, topology, transformer_architecture, 4, True, 2)


def get_tflops_bloom(iter_time_s: float, topology: Any, transformer_architecture: TransformerArchitectureConfig) -> float:
    """Megatron-paper count 96Bslh^2(1 + s/6h + V/16lh), with recompute factor when checkpointing."""
    a = transformer_architecture
    f = 3 if topology.config.activation_checkpointing_type == ActivationCheckpointingType.DISABLED else 4
    B, s, h, L, V = topology.config.global_batch_size, a.sequence_length, a.hidden_size, a.num_layers, a.vocab_size
    total = 24 * f * B * s * L * h * h + 4 * f * B * s * s * h * L + (2 + f) * B * s * h * V
    assert topology.config.world_size is not None
    return total / (iter_time_s * topology.config.world_size * 1e12)


def get_tflops_megatron(parameter_count: int, iter_time_s: float, topology: Any,
                        transformer_architecture: TransformerArchitectureConfig) -> float:
    a = transformer_architecture
    B = topology.config.global_batch_size
    ff = B * a.sequence_length * parameter_count * 6
    attn = B * a.sequence_length * a.sequence_length * a.hidden_size * a.num_layers * 60
    assert topology.config.world_size is not None
    return (ff + attn) / (iter_time_s * topology.config.world_size * 1e12)


class HardwareType(Enum):
    A100 = "a100"
    H100 = "h100"
    RTX3090 = "rtx3090"
    RTX4090 = "rtx4090"
    MI300X = "mi300x"
    MI355X = "mi355x"
    DEFAULT = "default"

    @property
    def max_tflops(self) -> float:
        """Dense 16-bit matrix peak in FLOP/s (never the 2:1-sparsity figures)."""
        return {"a100": 312e12, "h100": 989.4e12, "rtx3090": 35.58e12, "rtx4090": 82.58e12,
                "mi300x": 1307.4e12, "mi355x": 2516.6e12, "default": 0.0}[self.value]

    @classmethod
    def get_via_torch(cls) -> "HardwareType":
        if not torch.cuda.is_available():
            return cls.DEFAULT
        props = torch.cuda.get_device_properties(0)
        arch = getattr(props, "gcnArchName", "") or ""
        if arch.startswith("gfx950"):
            return cls.MI355X
        if arch.startswith("gfx942"):
            return cls.MI300X
        name = torch.cuda.get_device_name().replace(" ", "").lower().replace("nvidia", "")
        hit = next((x for x in cls if x != cls.DEFAULT and x.value in name), None)
        if hit is None:
            logger.warning(f"device {name} does not match any known HardwareType")
            return cls.DEFAULT
        return hit


def get_model_flop_utilization_palm(iter_time_s: float, parameter_count: int, topology: Any,
                                    transformer_architecture: TransformerArchitectureConfig) -> float:
    """PaLM MFU: tokens/s over peak/(6N + 12 L h s)."""
    a = transformer_architecture
    hw = HardwareType.get_via_torch()
    tokens_per_second = topology.config.global_batch_size * a.sequence_length / iter_time_s
    peak = hw.max_tflops * topology.config.world_size
    model_flops = 6 * parameter_count + 12 * a.num_layers * a.hidden_size * a.sequence_length
    return tokens_per_second / (peak / model_flops) if peak > 0 else 0.0


def get_tokens_per_second(iter_time_s: float, topology: Any, transformer_architecture: TransformerArchitectureConfig) -> float:
    return topology.config.global_batch_size * transformer_architecture.sequence_length / iter_time_s
