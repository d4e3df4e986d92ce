"""Forward-only pipeline schedule with two alternating buffers (reference ``pipeline_schedule/inference.py``)."""
from __future__ import annotations

from .base import PipelineScheduleBase
from .instructions import (
    InstructionBase,
    InstructionForwardPass,
    InstructionLoadMicroBatch,
    InstructionLoss,
    InstructionRecvActivation,
    InstructionSendActivation,
)


class PipelineScheduleInference(PipelineScheduleBase):
    def instructions(self) -> list[InstructionBase]:
        topo = self.topology
        rank = topo.pipe_parallel_rank
        even = rank % 2 == 0
        has_prev = self._is_valid_pipe_parallel_rank(topo.previous_pipe_parallel_rank)
        has_next = self._is_valid_pipe_parallel_rank(topo.next_pipe_parallel_rank)
        out: list[InstructionBase] = []
        for step in range(topo.config.gradient_accumulation_steps + topo.config.pipe_parallel_size - 1):
            mb = step - rank
            recv_buf, send_buf = (step % 2, (step + 1) % 2) if even else ((step + 1) % 2, step % 2)
            valid, next_valid = self._valid_micro_batch(mb), self._valid_micro_batch(mb - 1)
            if valid and (topo.is_first_pipe_parallel_rank or topo.is_last_pipe_parallel_rank):
                out.append(InstructionLoadMicroBatch(buffer_id=recv_buf, micro_batch_id=mb))
            send = [InstructionSendActivation(buffer_id=send_buf, micro_batch_id=mb)] if has_next and next_valid else []
            recv = [InstructionRecvActivation(buffer_id=recv_buf, micro_batch_id=mb)] if has_prev and valid else []
            out.extend(send + recv if even else recv + send)
            if valid:
                out.append(InstructionForwardPass(buffer_id=recv_buf, micro_batch_id=mb))
                if topo.is_last_pipe_parallel_rank:
                    out.append(InstructionLoss(buffer_id=recv_buf, micro_batch_id=mb))
        return out

    def required_buffer_count(self) -> int:
        return 2
