"""Compatibility alias: ``import scaling.core`` / ``scaling.transformer`` resolve to ``scaling_amd``.

Lets code written against the reference library (``from scaling.core import ...``) run unchanged
on the MI355X-native implementation.
"""
import importlib
import importlib.abc
import importlib.util
import sys


class _AliasFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    prefix = "scaling."

    def find_spec(self, fullname, path=None, target=None):  # noqa: ANN001
        if fullname.startswith(self.prefix):
            return importlib.util.spec_from_loader(fullname, self)
        return None

    def create_module(self, spec):  # noqa: ANN001
        real = importlib.import_module("scaling_amd." + spec.name[len(self.prefix):])
        sys.modules[spec.name] = real
        return real

    def exec_module(self, module):  # noqa: ANN001
        pass


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())
