from .trainer import BaseTrainer, DeterminedBaseTrainer
from .trainer_config import TrainerConfig

__all__ = ["BaseTrainer", "DeterminedBaseTrainer", "TrainerConfig"]
