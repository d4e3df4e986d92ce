"""Token samplers over logits [b, s, V] (reference ``transformer/inference/sample.py``)."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def sample_argmax(logits: torch.Tensor) -> torch.Tensor:
    return torch.argmax(logits, dim=-1)[:, -1]


def fast_multinomial(p: torch.Tensor) -> torch.Tensor:
    """One draw per row of ``p`` (inverse CDF; cheaper than torch.multinomial for a single sample)."""
    u = torch.rand(p.shape[:-1], device=p.device)[..., None]
    return (p.cumsum(-1) >= u).byte().argmax(-1)


def sample_temperature(logits: torch.Tensor, temperature: float = 1.0) -> torch.Tensor:
    return fast_multinomial(F.softmax(logits / temperature, dim=-1))[:, -1]


def top_k_transform(logits: torch.Tensor, k: int = 10) -> torch.Tensor:
    kth = torch.topk(logits, k)[0][..., -1, None]
    return logits.masked_fill(logits < kth, float("-inf"))


def top_p_transform(logits: torch.Tensor, threshold: float = 0.95) -> torch.Tensor:
    """Nucleus filtering of a 1-D logits vector: keep the smallest prefix of sorted tokens whose
    probability mass exceeds ``threshold`` (the first token is always kept)."""
    sorted_logits, order = torch.sort(logits, descending=True, dim=-1)
    cum = torch.cumsum(F.softmax(sorted_logits, dim=-1), dim=-1)
    drop = cum > threshold
    drop[1:] = drop[:-1].clone()
    drop[0] = False
    out = logits.clone()
    out[order[drop]] = float("-inf")
    return out
