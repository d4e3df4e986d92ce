from pathlib import Path
from typing import Optional

from pydantic import Field

from ..config import BaseConfig


class TrainerConfig(BaseConfig):
    save_dir: Optional[Path] = Field(None, description="directory for saving checkpoints")
    save_interval: Optional[int] = Field(None, description="save a checkpoint every 'save_interval' steps")
    load_dir: Optional[Path] = Field(None, description="directory for loading checkpoints")
    train_iterations: Optional[int] = Field(None, description="train for this number of iterations")
    assert_checkpoint_loaded: bool = Field(True, description="error out if a checkpoint could not be loaded")
    load_optimizer_states: bool = Field(True, description="load optimizer states on checkpoint load")
    delete_past_optimizer_states: bool = Field(
        True, description="delete optimizer states of older checkpoints after saving a new one (Determined only)"
    )
    load_context: bool = Field(True, description="load iterations / consumed samples / RNG on checkpoint load")
    allowed_missing_keys_in_checkpoint: Optional[list[str]] = Field(None, description="regexes of parameters that may be missing")
    allowed_unexpected_keys_in_checkpoint: Optional[list[str]] = Field(None, description="regexes of extra checkpoint keys to ignore")
    ignore_keys_in_checkpoint: Optional[list[str]] = Field(None, description="regexes of checkpoint keys not to load")
    merge_lora_after_loading_checkpoint: Optional[bool] = Field(False, description="merge LoRA weights after loading")
    seed: int = Field(42, description="")
    dataloader_num_workers: int = Field(0, description="")
    dataloader_pin_memory: bool = Field(True, description="")
    dataloader_prefetch_factor: Optional[int] = Field(None, description="")
    eval_iterations: int = Field(1, description="(not implemented in the reference either: one eval step)")
    eval_interval: Optional[int] = Field(None, description="evaluate every eval_interval steps")
    async_checkpointing: bool = Field(
        False,
        description="write checkpoint files from a background thread (state snapshotted to host memory first); "
        "'latest' is updated once every rank's files are complete, at the next save or the end of training",
    )
    hang_watchdog_seconds: Optional[float] = Field(
        None, description="MI355X addition: dump all thread stacks when a train step makes no progress for this many "
        "seconds (RCCL hang / stuck kernel diagnosis); None disables"
    )
    hang_watchdog_abort: bool = Field(False, description="exit the rank (code 124) after the hang dump so the launcher fails fast")
    separate_file_for_parameters: Optional[list[str]] = Field(
        None, description="create a separate checkpoint file for parameters matching these names"
    )
