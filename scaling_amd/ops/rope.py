"""Rotary position embedding (both conventions) with a HIP kernel (``csrc/kernels/swiglu_rope.hip``).

Inputs are token-major ``[T, heads, head_dim]`` views — typically strided slices of the fused QKV
GEMM output — and the kernel writes a contiguous rotated copy, so the attention kernel reads packed
heads.  Tables are fp32 ``[max_pos, rot_dim/2]``; the NeoX (rotate-half) table holds the cos/sin
values rounded through the model dtype, matching the reference's buffers (``rotary.py:93-108``);
the complex/interleaved table is fp32 as in ``rotary.py:45-90``.
"""
from __future__ import annotations

from typing import Any, Optional

import torch

from ._ext import ext, use_native


def rope_tables(dim: int, max_pos: int, base: float, interleaved: bool, dtype: torch.dtype, device: Any):
    inv_freq = 1.0 / (float(base) ** (torch.arange(0, dim, 2).float() / dim))
    t = torch.arange(max_pos).float()
    freqs = torch.outer(t, inv_freq)
    cos, sin = freqs.cos(), freqs.sin()
    if not interleaved and dtype != torch.float32:
        cos, sin = cos.to(dtype).float(), sin.to(dtype).float()
    return cos.contiguous().to(device), sin.contiguous().to(device)


def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: Optional[torch.Tensor],
                   rot_dim: int, seq_len: int, interleaved: bool) -> torch.Tensor:
    T = x.shape[0]
    p = pos.reshape(-1).long() if pos is not None else torch.arange(T, device=x.device) % seq_len
    c = cos[p][:, None, :]
    s = sin[p][:, None, :]
    xf = x.float()
    rot, rest = xf[..., :rot_dim], xf[..., rot_dim:]
    if interleaved:
        x0, x1 = rot[..., 0::2], rot[..., 1::2]
        o0, o1 = x0 * c - x1 * s, x1 * c + x0 * s
        out = torch.stack([o0, o1], dim=-1).flatten(-2)
    else:
        h = rot_dim // 2
        x0, x1 = rot[..., :h], rot[..., h:]
        out = torch.cat([x0 * c - x1 * s, x1 * c + x0 * s], dim=-1)
    return torch.cat([out, rest], dim=-1).to(x.dtype)


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, x, cos, sin, pos, rot_dim, seq_len, interleaved):  # type: ignore[override]
        ctx.save_for_backward(cos, sin, pos)
        ctx.cfg = (rot_dim, seq_len, interleaved)
        return ext().rope(x, cos, sin, pos, rot_dim, seq_len, interleaved, False)

    @staticmethod
    def backward(ctx: Any, dy: torch.Tensor):  # type: ignore[override]
        cos, sin, pos = ctx.saved_tensors
        rot_dim, seq_len, interleaved = ctx.cfg
        dx = ext().rope(dy.contiguous(), cos, sin, pos, rot_dim, seq_len, interleaved, True)
        return dx, None, None, None, None, None, None


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: Optional[torch.Tensor], rot_dim: int,
               seq_len: int, interleaved: bool) -> torch.Tensor:
    """x: [T, heads, head_dim]; pos: [T] absolute positions or None (position = t % seq_len)."""
    if use_native(x):
        if pos is not None:
            pos = pos.reshape(-1).long().contiguous()
        return _Rope.apply(x, cos, sin, pos, rot_dim, seq_len, interleaved)
    return rope_reference(x, cos, sin, pos, rot_dim, seq_len, interleaved)
