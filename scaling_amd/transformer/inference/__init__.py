from .inference_model import CompletionOutput, TransformerInferenceModule
from .sample import fast_multinomial, sample_argmax, sample_temperature, top_k_transform, top_p_transform

__all__ = [
    "CompletionOutput",
    "TransformerInferenceModule",
    "fast_multinomial",
    "sample_argmax",
    "sample_temperature",
    "top_k_transform",
    "top_p_transform",
]
