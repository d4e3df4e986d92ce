from .indexed_dataset import (
    IndexedCachedDataset,
    IndexedDataset,
    MMapIndexedDataset,
    MMapIndexedDatasetBuilder,
    get_indexed_dataset_,
    infer_dataset_impl,
    make_builder,
    make_dataset,
)

__all__ = [
    "IndexedCachedDataset",
    "IndexedDataset",
    "MMapIndexedDataset",
    "MMapIndexedDatasetBuilder",
    "get_indexed_dataset_",
    "infer_dataset_impl",
    "make_builder",
    "make_dataset",
]
