from .base_dataset import BaseDataset, BaseDatasetBatch, BaseDatasetItem
from .base_layer_io import BaseLayerIO
from .blended_dataset import BaseBlendedDataset, weights_by_num_docs, weights_examples_proportional
from .blended_dataset_config import BlendedDatasetConfig
from .broadcast_data import broadcast_data
from .dataloader import DataLoader, RandomSampler
from .file_dataset import FileDataset
from .file_handles import FileHandle, RetryableException
from .memory_map import MemoryMapDataset, MemoryMapDatasetBuilder

__all__ = [
    "BaseBlendedDataset",
    "BaseDataset",
    "BaseDatasetBatch",
    "BaseDatasetItem",
    "BaseLayerIO",
    "BlendedDatasetConfig",
    "DataLoader",
    "FileDataset",
    "FileHandle",
    "MemoryMapDataset",
    "MemoryMapDatasetBuilder",
    "RandomSampler",
    "RetryableException",
    "broadcast_data",
    "weights_by_num_docs",
    "weights_examples_proportional",
]
