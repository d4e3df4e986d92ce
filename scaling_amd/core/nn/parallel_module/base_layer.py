"""Pipeline layer interface (reference ``parallel_module/base_layer.py:16-115``)."""
from __future__ import annotations

from abc import abstractmethod
from typing import Any, Generic, TypeVar

import torch

from ...data import BaseDatasetBatch, BaseLayerIO

BaseLossInputGeneric = TypeVar("BaseLossInputGeneric")
BaseLossOutputGeneric = TypeVar("BaseLossOutputGeneric")
BaseDatasetBatchGeneric = TypeVar("BaseDatasetBatchGeneric", bound=BaseDatasetBatch)
BaseLayerInputGeneric = TypeVar("BaseLayerInputGeneric")
BaseLayerOutputGeneric = TypeVar("BaseLayerOutputGeneric", bound=BaseLayerIO)
BaseLayerLastLayerOutputGeneric = TypeVar("BaseLayerLastLayerOutputGeneric", bound=BaseLayerIO)


class BaseLayer(torch.nn.Module, Generic[BaseLayerInputGeneric, BaseLayerOutputGeneric, BaseLayerLastLayerOutputGeneric]):
    @abstractmethod
    def forward(self, x: BaseLayerInputGeneric) -> BaseLayerOutputGeneric:
        raise NotImplementedError

    @staticmethod
    @abstractmethod
    def input_to_tuple(input: BaseLayerInputGeneric) -> tuple[Any, ...]:
        """Layer input -> tuple (pipeline p2p / activation checkpointing)."""
        raise NotImplementedError

    @staticmethod
    @abstractmethod
    def tuple_to_input(d: tuple[Any, ...]) -> BaseLayerInputGeneric:
        raise NotImplementedError

    @staticmethod
    @abstractmethod
    def output_to_tuple(output: BaseLayerOutputGeneric) -> tuple[Any, ...]:
        raise NotImplementedError

    @staticmethod
    @abstractmethod
    def tuple_to_last_stage_activation(d: tuple[Any, ...]) -> BaseLayerLastLayerOutputGeneric:
        raise NotImplementedError

    def _forward_tuple_input(self, *args: Any) -> Any:
        return self(self.tuple_to_input(tuple(args)))
