"""Llama-family architecture presets expressed in the reference's ``TransformerArchitectureConfig``
schema (``transformer/context/config.py``): pre-RMSNorm, RoPE, SwiGLU, untied head, no biases,
optional grouped-query attention.  ``llama2_7b`` is the headline benchmark shape."""
from __future__ import annotations

from typing import Any, Optional

_PRESETS: dict[str, dict[str, Any]] = {
    # h, layers, heads, kv heads (GQA variant of the benchmark), SwiGLU width
    "llama2_7b": dict(hidden_size=4096, num_layers=32, num_attention_heads=32, kv_heads=8, ffn=11008),
    "llama2_7b_mha": dict(hidden_size=4096, num_layers=32, num_attention_heads=32, kv_heads=32, ffn=11008),
    "llama2_13b": dict(hidden_size=5120, num_layers=40, num_attention_heads=40, kv_heads=40, ffn=13824),
    "llama2_70b": dict(hidden_size=8192, num_layers=80, num_attention_heads=64, kv_heads=8, ffn=28672),
    "llama_1b": dict(hidden_size=2048, num_layers=16, num_attention_heads=16, kv_heads=4, ffn=5632),
    "llama_tiny": dict(hidden_size=256, num_layers=2, num_attention_heads=4, kv_heads=2, ffn=688),
    # llama_tiny with every GEMM dimension a multiple of 256 (ffn 768): every weight gradient tiles onto the
    # hand-written HIP kernel and every dgrad onto the W^T cache (SCALING_AMD_DGRAD_WT=all; tests/test_gpu_e2e.py)
    "llama_tiny_r256": dict(hidden_size=256, num_layers=2, num_attention_heads=4, kv_heads=2, ffn=768),
}


def preset_names() -> list[str]:
    return sorted(_PRESETS)


def llama_architecture(name: str = "llama2_7b", sequence_length: int = 4096, vocab_size: int = 32000,
                       precision: str = "bfloat16", kv_heads: Optional[int] = None, flash_attention: bool = True,
                       **overrides: Any) -> dict[str, Any]:
    """Returns a ``transformer_architecture`` config dict for the named preset."""
    p = _PRESETS[name]
    h, ffn = p["hidden_size"], p["ffn"]
    kv = p["kv_heads"] if kv_heads is None else kv_heads
    arch: dict[str, Any] = {
        "vocab_size": vocab_size,
        "hidden_size": h,
        "num_layers": p["num_layers"],
        "num_attention_heads": p["num_attention_heads"],
        "attention_num_kv_heads": None if kv == p["num_attention_heads"] else kv,
        "attention_qkv_in_one": kv == p["num_attention_heads"],
        "sequence_length": sequence_length,
        "norm_type": "rms",
        "layernorm": {"optimization_type": "fused", "layernorm_epsilon": 1e-5},
        "relative_position_embedding_type": "rotary_complex",
        "rotary_embedding_base": 10000,
        "mlp_type": "swiglu",
        "mlp_factor": ffn / h,
        "attention_bias": False,
        "mlp_bias": False,
        "weight_tying": False,
        "precision": precision,
        "masked_softmax": {"kernel": "flash_attention" if flash_attention else "torch"},
        "causal": True,
    }
    assert int(h * arch["mlp_factor"]) == ffn
    arch.update(overrides)
    return arch
