"""Dataset interfaces (reference ``src/scaling/core/data/base_dataset.py:12-108``)."""
from __future__ import annotations

from abc import abstractmethod
from typing import Any, Generic, Optional, TypeVar

import torch

from .base_layer_io import BaseLayerIO

TBaseDatasetBatch = TypeVar("TBaseDatasetBatch", bound="BaseDatasetBatch")


class BaseDatasetItem:
    """Base class for dataset items."""


class BaseDatasetBatch(BaseLayerIO):
    """Base class for batches; ``only_inputs``/``only_targets`` drop what a pipeline stage does not need."""

    @abstractmethod
    def only_inputs(self: TBaseDatasetBatch) -> TBaseDatasetBatch:
        return self

    @abstractmethod
    def only_targets(self: TBaseDatasetBatch) -> TBaseDatasetBatch:
        return self


BaseDatasetItemGeneric = TypeVar("BaseDatasetItemGeneric", bound=BaseDatasetItem)
BaseDatasetBatchBeforeSyncGeneric = TypeVar("BaseDatasetBatchBeforeSyncGeneric", bound=BaseDatasetBatch)
BaseDatasetBatchGeneric = TypeVar("BaseDatasetBatchGeneric", bound=BaseDatasetBatch)


class BaseDataset(
    torch.utils.data.Dataset,
    Generic[BaseDatasetItemGeneric, BaseDatasetBatchBeforeSyncGeneric, BaseDatasetBatchGeneric],
):
    def __init__(self, seed: int, shuffle: bool = True) -> None:
        self.seed: Optional[int] = None
        self.set_seed(seed=seed, shuffle=shuffle)

    @abstractmethod
    def ident(self) -> str:
        raise NotImplementedError

    @abstractmethod
    def __len__(self) -> int:
        raise NotImplementedError

    @abstractmethod
    def __getitem__(self, index: int) -> BaseDatasetItemGeneric:
        raise NotImplementedError

    @abstractmethod
    def set_seed(self, seed: int, shuffle: bool = True) -> None:
        raise NotImplementedError

    @abstractmethod
    def collate(self, batch: list[BaseDatasetItemGeneric]) -> BaseDatasetBatchBeforeSyncGeneric:
        raise NotImplementedError

    @staticmethod
    @abstractmethod
    def sync_batch_to_model_parallel(topology: Any, batch: Optional[BaseDatasetBatchBeforeSyncGeneric]) -> Any:
        raise NotImplementedError

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}"
