"""Race-check forensics: stream-ordered checksums of the gradients flowing through named points of the backward.

``enable(records)`` turns probing on: every ``probe(name, t)`` on a tensor that requires grad then registers a hook
that appends ``(name, tensor([sum, sum of squares]))`` (float64, on the device, no host sync) to ``records`` when the
backward reaches ``t``, so ``records`` lists the gradients in backward execution order.  Two runs that should be
bit-identical are compared entry by entry (``tools/race_trace.py``): the first differing entry names the op that ran
between it and the previous entry.  Off (the default) ``probe`` is a dictionary lookup."""
from __future__ import annotations

from typing import Any, Optional

import torch

_records: Optional[list] = None


def enable(records: list) -> None:
    global _records
    _records = records


def disable() -> None:
    global _records
    _records = None


def probe(name: str, t: Any) -> Any:
    rec = _records
    if rec is not None and torch.is_tensor(t) and t.requires_grad and t.is_floating_point():
        t.register_hook(lambda g, n=name: rec.append(
            (n, torch.stack([g.double().sum(), (g.double() * g.double()).sum()]))))
    return t


def record(name: str, *tensors: Any) -> None:
    """Appends ``(name, [sum, sum of squares] per tensor)`` of arbitrary tensors (saved activations, buffers) at this
    point of the stream, when probing is on: e.g. an op's saved inputs once in its forward and again at the start of
    its backward, so a change in between (something writing into memory it does not own) shows up as a differing
    entry."""
    rec = _records
    if rec is None:
        return
    vals = []
    for t in tensors:
        if torch.is_tensor(t) and t.numel():
            d = t.detach().double()
            vals += [d.sum(), (d * d).sum()]
    if vals:
        rec.append((name, torch.stack(vals)))


def enabled() -> bool:
    return _records is not None


def record_values(name: str, t: Any) -> None:
    """Appends ``(name, t)`` itself (a small float64 vector of diagnostic values) when probing is on."""
    rec = _records
    if rec is not None and torch.is_tensor(t):
        rec.append((name, t.detach().double().reshape(-1)))
