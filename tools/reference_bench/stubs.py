"""Import stubs for the reference's optional integrations that this image does not ship (wandb, determined,
torchvision, tensorboard and torch's tensorboard writer).  Only used by ``ref_bench.py`` to import the unmodified reference for a
same-hardware baseline: any attribute of a stubbed module is an inert placeholder class, and nothing in the
benchmarked path (training step of the 7B shape) calls into them."""
from __future__ import annotations

import importlib.abc
import importlib.machinery
import sys
import types

STUBBED = ("wandb", "determined", "torchvision", "tensorboard", "torch.utils.tensorboard")


class _PlaceholderMeta(type):
    def __getattr__(cls, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Placeholder()


class _Placeholder(metaclass=_PlaceholderMeta):
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return self

    def __getattr__(self, name):
        return _Placeholder()


class _StubModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        cls = type(name, (_Placeholder,), {})
        setattr(self, name, cls)
        return cls


class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if any(fullname == s or fullname.startswith(s + ".") for s in STUBBED):
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _StubModule(spec.name)
        m.__path__ = []  # package: submodules resolve through this finder too
        m.__version__ = "99.0"
        return m

    def exec_module(self, module):
        pass


def install() -> None:
    if not any(isinstance(f, _Finder) for f in sys.meta_path):
        sys.meta_path.insert(0, _Finder())
