from .base_layer import BaseLayer
from .buffers import Buffers, BufferType
from .communicator import ModelParallelCommunicator, PipeCommunicator
from .inference_module import HiddenStateRecorder, InferenceModule, RecorderSetting
from .layer_spec import LayerSpec, TiedLayerSpec
from .parallel_module import EvaluationStepOutput, ParallelModule, TrainStepOutput
from .partitioned_module import PipePartitionedModule, key_match
from .pipeline_partitioning import (
    PipePartitionCoordinates,
    pipe_partition_balanced,
    pipe_partition_from_indices,
    pipe_partition_uniform,
)
from .tied_layer_index import TiedLayerIndex

__all__ = [
    "BaseLayer",
    "BufferType",
    "Buffers",
    "EvaluationStepOutput",
    "HiddenStateRecorder",
    "InferenceModule",
    "LayerSpec",
    "ModelParallelCommunicator",
    "ParallelModule",
    "PipeCommunicator",
    "PipePartitionCoordinates",
    "PipePartitionedModule",
    "RecorderSetting",
    "TiedLayerIndex",
    "TiedLayerSpec",
    "TrainStepOutput",
    "key_match",
    "pipe_partition_balanced",
    "pipe_partition_from_indices",
    "pipe_partition_uniform",
]
