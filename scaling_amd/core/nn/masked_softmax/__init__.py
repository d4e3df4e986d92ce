from .masked_softmax import MaskedSoftmax, MaskedSoftmaxTorch
from .masked_softmax_config import MaskedSoftmaxConfig, MaskedSoftmaxKernel

__all__ = ["MaskedSoftmax", "MaskedSoftmaxConfig", "MaskedSoftmaxKernel", "MaskedSoftmaxTorch"]
