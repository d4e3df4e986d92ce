from pydantic import Field

from ..config import BaseConfig


class RotaryConfig(BaseConfig):
    dimensions: int = Field(0, description="number of rotated dimensions per head")
    base: int = Field(10000, description="rotary base")
    max_seq_length: int = Field(2048, description="size of the precomputed position table")
