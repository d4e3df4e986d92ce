"""Loader for the in-tree HIP extension (``scaling_amd._C``).

Policy: a GPU tensor ALWAYS goes through the HIP kernels; if the extension is missing on a GPU box the
op raises (no silent eager fallback).  CPU tensors (gloo CI, numerics oracles) use the pure-torch
reference implementations that live next to each op.
"""
from __future__ import annotations

import importlib.util
import os
import sys
from types import ModuleType
from typing import Optional

import torch

_EXT: Optional[ModuleType] = None


def ext() -> ModuleType:
    global _EXT
    if _EXT is None:
        variant = os.environ.get("SCALING_AMD_EXT_SO")
        if variant:  # a build variant for an A/B (scaling_amd/_build.py: SCALING_AMD_FILE_FLAGS / _BUILD_OUT)
            spec = importlib.util.spec_from_file_location("scaling_amd._C", variant)
            if spec is None or spec.loader is None:
                raise RuntimeError(f"SCALING_AMD_EXT_SO={variant}: not a loadable extension")
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["scaling_amd._C"] = mod
            _EXT = mod
            return mod
        try:
            from scaling_amd import _C  # type: ignore[attr-defined]
        except ImportError as e:  # pragma: no cover - depends on build state
            raise RuntimeError(
                "scaling_amd HIP extension is not built (python -c 'import __graft_entry__ as g; g.build()' "
                "or python -m scaling_amd._build)"
            ) from e
        _EXT = _C
    return _EXT


def use_native(*tensors: torch.Tensor) -> bool:
    return any(t is not None and t.is_cuda for t in tensors)


def available() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False
