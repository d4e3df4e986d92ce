from pydantic import Field

from ..config import BaseConfig


class LossScalerConfig(BaseConfig):
    """Dynamic loss scaling for fp16 training (reference ``loss_scaler_config.py:13``)."""

    enable: bool = Field(False, description="")
    initial_scale: float = Field(2.0**32, description="Initial loss scale")
    window: int = Field(1000, description="steps without overflow before the scale grows")
    hysteresis: float = Field(2, description="overflows tolerated before the scale shrinks")
    consecutive_hysteresis: bool = Field(False, description="reset hysteresis on every non-overflow step")
    min_scale: float = Field(1.0, description="")
    factor: float = Field(2.0, description="")
