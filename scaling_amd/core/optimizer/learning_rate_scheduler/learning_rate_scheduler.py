"""Warmup + constant/linear/cosine decay (semantics of reference ``learning_rate_scheduler.py:18-89``)."""
import math

from .learning_rate_scheduler_config import LearningRateDecayStyle, LearningRateSchedulerConfig


class LearningRateScheduler:
    def __init__(self, config: LearningRateSchedulerConfig):
        self.config = config

    def get_lr(self, step_index: int) -> float:
        c = self.config
        if c.learning_rate_warmup_steps > 0 and step_index <= c.learning_rate_warmup_steps:
            return c.learning_rate * float(step_index) / float(c.learning_rate_warmup_steps)
        if c.learning_rate_decay_style == LearningRateDecayStyle.CONSTANT:
            return c.learning_rate
        if step_index > c.learning_rate_decay_iters:
            return c.learning_rate_minimum
        ratio = float(step_index - c.learning_rate_warmup_steps) / float(
            c.learning_rate_decay_iters - c.learning_rate_warmup_steps
        )
        assert 0.0 <= ratio <= 1.0
        if c.learning_rate_decay_style == LearningRateDecayStyle.LINEAR:
            coeff = 1.0 - ratio
        else:
            coeff = 0.5 * (math.cos(math.pi * ratio) + 1.0)
        return c.learning_rate_minimum + coeff * (c.learning_rate - c.learning_rate_minimum)
