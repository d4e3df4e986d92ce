from .finetuning_chat_dataset import FinetuningChatBlendedDataset, FinetuningChatDataset
from .finetuning_text_dataset import FinetuningTextBlendedDataset, FinetuningTextDataset
from .inference_settings import Control, InferenceSettings, InferenceSuppressionParameters
from .legacy_blended_dataset import LegacyBlendedDataset
from .text_dataset import TextBlendedDataset, TextDataset
from .text_dataset_batch import TextDatasetBatch, TextDatasetBatchBeforeSync
from .text_dataset_item import TextDatasetItem
from .utils import get_cumulative_seq_lengths, get_position_ids

__all__ = [
    "Control",
    "FinetuningChatBlendedDataset",
    "FinetuningChatDataset",
    "FinetuningTextBlendedDataset",
    "FinetuningTextDataset",
    "LegacyBlendedDataset",
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
