import math
from enum import Enum

from pydantic import Field

from ..config import BaseConfig


class LoRAModuleType(Enum):
    QUERY = "query"
    KEY = "key"
    VALUE = "value"
    DENSE = "dense"


class LoRaConfig(BaseConfig):
    name: str = Field(default="lora", description="")
    rank: int = Field(default=64, description="Intrinsic rank of the LoRA adapter over all heads.")
    parallel_modules: list[LoRAModuleType] = Field(
        default=[LoRAModuleType.DENSE, LoRAModuleType.KEY, LoRAModuleType.VALUE, LoRAModuleType.QUERY],
        description="Linear layers that receive a parallel LoRA adapter",
    )
    dropout: float = Field(default=0.0, description="dropout probability inside LoRA")
    alpha: int = Field(default=1, description="LoRA scaling alpha (scaling = alpha / rank)")
    bias: bool = Field(default=False, description="use bias in LoRA modules")
    kaiming_a: float = Field(default=math.sqrt(5), description="kaiming 'a' for the A matrix init")
