"""MI355X (gfx950) HIP kernels with autograd wrappers.

Every op dispatches GPU tensors to the in-tree HIP extension and CPU tensors to a pure-torch
reference implementation (used by CPU/gloo tests and as the numerical oracle in GPU tests).
"""
from . import attention, embedding, norm, optim, rope, swiglu, xent  # noqa: F401
from ._ext import available, ext, use_native  # noqa: F401
