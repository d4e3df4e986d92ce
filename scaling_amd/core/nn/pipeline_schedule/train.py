"""1F1B training schedule (reference ``pipeline_schedule/train.py:32-174``; DeepSpeed TrainSchedule order).

Steps alternate forward/backward by parity of (step, stage) so neighbouring stages always pair a
send with the matching receive (deadlock-free with blocking p2p); the instruction order is kept
identical to the reference because loss equality across layouts depends on it.
"""
from __future__ import annotations

from .base import PipelineScheduleBase
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
)


class PipelineScheduleTrain(PipelineScheduleBase):
    def _step_to_micro_batch(self, step: int) -> tuple[int, bool]:
        r = self.topology.pipe_parallel_rank
        pp = self.topology.config.pipe_parallel_size
        forward = (step % 2) == (r % 2)
        half = step // 2 if step % 2 == 0 else (step - 1) // 2
        if forward:
            return half - r // 2, True
        if step % 2 == 0:  # even step, odd stage
            return half - pp + (r + 1) // 2, False
        return half - pp + 1 + r // 2, False  # odd step, even stage

    def instructions(self) -> list[InstructionBase]:
        topo = self.topology
        acc, pp = topo.config.gradient_accumulation_steps, topo.config.pipe_parallel_size
        has_prev = self._is_valid_pipe_parallel_rank(topo.previous_pipe_parallel_rank)
        has_next = self._is_valid_pipe_parallel_rank(topo.next_pipe_parallel_rank)
        io_stage = topo.pipe_parallel_rank in (0, pp - 1)
        total = 2 * (acc + pp - 1)
        out: list[InstructionBase] = []
        prev = -1
        for step in range(total):
            mb, fwd = self._step_to_micro_batch(step)
            valid, prev_valid = self._valid_micro_batch(mb), self._valid_micro_batch(prev)
            buf = self._buffer_idx(mb) if valid else None
            pbuf = self._buffer_idx(prev) if prev_valid else None
            if fwd:
                if valid and has_prev:
                    out.append(InstructionRecvActivation(buffer_id=buf, micro_batch_id=mb))
                if prev_valid and has_prev:
                    out.append(InstructionSendGrad(buffer_id=pbuf, micro_batch_id=prev))
            else:
                if prev_valid and has_next:
                    out.append(InstructionSendActivation(buffer_id=pbuf, micro_batch_id=prev))
                if valid and has_next:
                    out.append(InstructionRecvGrad(buffer_id=buf, micro_batch_id=mb))
            if io_stage and fwd and valid:
                out.append(InstructionLoadMicroBatch(buffer_id=buf, micro_batch_id=mb))
            if valid:
                if fwd:
                    out.append(InstructionForwardPass(buffer_id=buf, micro_batch_id=mb))
                    if topo.is_last_pipe_parallel_rank:
                        out.append(InstructionLoss(buffer_id=buf, micro_batch_id=mb, is_first_pass=True))
                else:
                    out.append(InstructionBackwardPass(buffer_id=buf, micro_batch_id=mb))
            if step == total - 1:
                out.append(InstructionReduceTiedGrads())
                out.append(InstructionOptimizerStep())
            prev = mb
        return out

    def required_buffer_count(self) -> int:
        n = min(
            self.topology.config.pipe_parallel_size - self.topology.pipe_parallel_rank + 1,
            self.topology.config.gradient_accumulation_steps,
        )
        return max(2, n)

    def _buffer_idx(self, micro_batch_id: int) -> int:
        assert self._valid_micro_batch(micro_batch_id)
        return micro_batch_id % self.required_buffer_count()
