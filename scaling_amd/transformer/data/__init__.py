from .inference_settings import Control, InferenceSettings, InferenceSuppressionParameters
from .text_dataset import TextBlendedDataset, TextDataset
from .text_dataset_batch import TextDatasetBatch, TextDatasetBatchBeforeSync
from .text_dataset_item import TextDatasetItem
from .utils import get_cumulative_seq_lengths, get_position_ids

__all__ = [
    "Control",
    "InferenceSettings",
    "InferenceSuppressionParameters",
    "TextBlendedDataset",
    "TextDataset",
    "TextDatasetBatch",
    "TextDatasetBatchBeforeSync",
    "TextDatasetItem",
    "get_cumulative_seq_lengths",
    "get_position_ids",
]
