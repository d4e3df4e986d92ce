from .base import DEPENDENCY_MAP, PipelineScheduleBase, SimulationEngine
from .inference import PipelineScheduleInference
from .instructions import (
    InstructionBackwardPass,
    InstructionBase,
    InstructionForwardPass,
    InstructionLoadMicroBatch,
    InstructionLoss,
    InstructionOptimizerStep,
    InstructionRecvActivation,
    InstructionRecvGrad,
    InstructionReduceTiedGrads,
    InstructionSendActivation,
    InstructionSendGrad,
    InstructionStoreMicroBatch,
)
from .train import PipelineScheduleTrain

__all__ = [
    "DEPENDENCY_MAP",
    "InstructionBackwardPass",
    "InstructionBase",
    "InstructionForwardPass",
    "InstructionLoadMicroBatch",
    "InstructionLoss",
    "InstructionOptimizerStep",
    "InstructionRecvActivation",
    "InstructionRecvGrad",
    "InstructionReduceTiedGrads",
    "InstructionSendActivation",
    "InstructionSendGrad",
    "InstructionStoreMicroBatch",
    "PipelineScheduleBase",
    "PipelineScheduleInference",
    "PipelineScheduleTrain",
    "SimulationEngine",
]
