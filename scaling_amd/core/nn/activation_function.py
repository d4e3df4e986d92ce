"""Activation functions of the MLP blocks (reference ``nn/activation_function.py``): the config enum is
kept, the callables run the HIP elementwise kernels on GPU tensors (``scaling_amd.ops.elementwise``)."""
from __future__ import annotations

from enum import Enum
from functools import partial
from typing import Callable

import torch

from ...ops.elementwise import activation


class ActivationFunction(Enum):
    GELU = "gelu"
    SILU = "silu"


_KIND = {ActivationFunction.GELU: "gelu", ActivationFunction.SILU: "silu"}


def get_activation_function(activation_function: ActivationFunction) -> Callable[[torch.Tensor], torch.Tensor]:
    try:
        return partial(activation, kind=_KIND[ActivationFunction(activation_function)])
    except KeyError:
        raise NotImplementedError(str(activation_function)) from None
