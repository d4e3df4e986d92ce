"""Checkpoint loading without executing code from the file.

Every ``.pt`` file of a checkpoint (model, optimizer, context) is read with ``weights_only=True``.
The only non-tensor globals the framework's own files hold are the numpy RNG state of the context
(``np.random.get_state()``: an ndarray + dtype), which are allow-listed here; python sets, tuples,
dicts, dtypes and python RNG state are covered by the weights-only unpickler itself.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Union

import numpy as np
import torch


def _numpy_globals() -> list[Any]:
    out: list[Any] = [np.ndarray, np.dtype]
    for mod in ("numpy._core.multiarray", "numpy.core.multiarray"):
        try:
            m = __import__(mod, fromlist=["_reconstruct"])
            out.append(m._reconstruct)
        except (ImportError, AttributeError):
            continue
    out.extend(type(np.dtype(t)) for t in ("uint32", "int64", "float64"))
    return out


def safe_load(path: Union[str, Path], map_location: Any = None) -> Any:
    with torch.serialization.safe_globals(_numpy_globals()):
        return torch.load(str(path), map_location=map_location, weights_only=True)
