"""Pipeline instructions (reference ``pipeline_schedule/instructions.py:5-61``)."""
from typing import NamedTuple, Optional


class InstructionBase(NamedTuple):
    buffer_id: Optional[int] = None
    micro_batch_id: Optional[int] = None
    is_first_pass: Optional[bool] = None

    @property
    def name(self) -> str:
        return self.__class__.__name__


class InstructionOptimizerStep(InstructionBase):
    pass


class InstructionReduceTiedGrads(InstructionBase):
    pass


class InstructionStoreMicroBatch(InstructionBase):
    pass


class InstructionLoadMicroBatch(InstructionBase):
    pass


class InstructionForwardPass(InstructionBase):
    pass


class InstructionLoss(InstructionBase):
    pass


class InstructionBackwardPass(InstructionBase):
    pass


class InstructionSendActivation(InstructionBase):
    pass


class InstructionRecvActivation(InstructionBase):
    pass


class InstructionSendGrad(InstructionBase):
    pass


class InstructionRecvGrad(InstructionBase):
    pass
