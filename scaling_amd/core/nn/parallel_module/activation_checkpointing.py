"""Activation checkpointing that also replays the model-parallel-constant RNG stream.

Parity: reference ``activation_checkpointing.py:72-190`` (non-reentrant checkpoint that snapshots
and restores the Topology RNG tracker so recomputed dropout matches).  Built on the public
``torch.utils.checkpoint(use_reentrant=False, context_fn=...)`` API; torch's own
``preserve_rng_state`` covers the global CPU/HIP generators.
"""
from __future__ import annotations

import contextlib
from typing import Any, Callable, Iterator

import torch
from torch.utils.checkpoint import checkpoint

from ....ops.attention import AttentionStash, attention_stash


def _tracker_contexts(topology: Any, keep_attention: bool = False, keep_gemms: bool = False) -> tuple:
    tracker = getattr(topology, "_model_parallel_constant_rng", None)
    saved: dict[str, Any] = {}
    # lives as long as this checkpoint's frame: recorded in the forward, drained by the recompute
    stash = AttentionStash(keep_gemms=keep_gemms) if (keep_attention or keep_gemms) else None

    @contextlib.contextmanager
    def forward_ctx() -> Iterator[None]:
        if tracker is not None:
            saved["state"] = tracker.state.clone()
        with attention_stash(stash, "record"):
            yield

    @contextlib.contextmanager
    def recompute_ctx() -> Iterator[None]:
        with attention_stash(stash, "replay"):
            if tracker is None or "state" not in saved:
                yield
                return
            current = tracker.state
            tracker.state = saved["state"].clone()
            try:
                yield
            finally:
                tracker.state = current

    return forward_ctx(), recompute_ctx()


def checkpoint_with_rng(function: Callable[..., Any], topology: Any, preserve_rng_state: bool, *args: Any,
                        keep_attention: bool = False, keep_gemms: bool = False) -> Any:
    """Non-reentrant checkpoint of ``function(*args)`` that replays the TP-constant RNG stream; with
    ``keep_attention`` the flash-attention outputs of the first forward are kept and reused by the recompute, with
    ``keep_gemms`` also every linear layer's GEMM output (selective recompute of the element-wise work only)."""
    return checkpoint(
        function,
        *args,
        use_reentrant=False,
        preserve_rng_state=preserve_rng_state,
        context_fn=lambda: _tracker_contexts(topology, keep_attention, keep_gemms),
    )


# reference-compatible name
_checkpoint_without_reentrant = checkpoint_with_rng
