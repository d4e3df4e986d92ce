from pathlib import Path
from typing import Optional

from pydantic import Field

from ..config import BaseConfig


class BlendedDatasetConfig(BaseConfig):
    """Blending of several datasets (field-compatible with reference ``blended_dataset_config.py``)."""

    weight_by_num_documents: bool = Field(
        True, description="weights from a multinomial over the datasets' document counts (overrides `weights`)"
    )
    weighted_sampler_alpha: float = Field(1.0, description="alpha of weight_by_num_documents")
    weights: Optional[list[float]] = Field(None, description="explicit dataset weights")
    weight_examples_proportional: bool = Field(False, description="examples-proportional mixing (T5)")
    ep_maximum: Optional[int] = Field(None, description="rate limit K for examples-proportional mixing")
    ep_temperature: float = Field(1.0, description="temperature for examples-proportional mixing")
    minimum_dataset_size: int = Field(0, description="Minimal size of the dataset.")
    cache_directory: Optional[Path] = Field(None, description="directory to cache the blended dataset index")
    shuffle_dataset_indices: bool = Field(False, description="shuffle after blended index creation")
    load_dataset_indices_to_memory: bool = Field(False, description="load indices to memory rather than mmap")
