"""Infinite, resumable, data-parallel-strided data loader (reference ``core/data/dataloader.py:18-162``).

Sample order is identical to the reference: epoch = consumed // usable_total, indices
``k * dp + dp_rank + consumed_in_epoch``, the dataset is re-seeded with ``seed + epoch`` at every
epoch start, incomplete micro batches are dropped — so a resumed run sees exactly the same data.
"""
from __future__ import annotations

from typing import Any, Generator, Optional

import torch

from ..logging import logger
from .base_dataset import BaseDataset


class RandomSampler:
    def __init__(self, dataset: BaseDataset, seed: int, consumed_samples: int, topology: Any, shuffle: bool = True):
        self.dataset = dataset
        self.seed = seed
        self.consumed_samples = consumed_samples
        self.topology = topology
        self.shuffle = shuffle
        cfg = topology.config
        self.total_samples = len(dataset)
        self.total_micro_batches = len(dataset) // cfg.micro_batch_size
        self.total_micro_batches_per_data_parallel = self.total_micro_batches // cfg.data_parallel_size
        self.usable_total_samples = (
            self.total_micro_batches_per_data_parallel * cfg.micro_batch_size * cfg.data_parallel_size
        )
        assert self.usable_total_samples > 0, (
            "not usable samples; the dataset is too small for the data parallel size and micro batch size"
        )

    def __len__(self) -> int:
        return self.total_micro_batches

    def __iter__(self) -> Generator[list[int], None, None]:
        cfg = self.topology.config
        epoch = self.consumed_samples // self.usable_total_samples
        in_epoch = self.consumed_samples % self.usable_total_samples
        remaining = self.usable_total_samples - in_epoch
        logger.info(f"creating new dataset shuffle index for epoch {epoch} (consumed in epoch {in_epoch})")
        self.dataset.set_seed(seed=self.seed + epoch, shuffle=self.shuffle)
        dp = cfg.data_parallel_size
        idx = (torch.arange(0, remaining // dp, dtype=torch.long) * dp + self.topology.data_parallel_rank + in_epoch).tolist()
        assert len(idx) % cfg.micro_batch_size == 0, "dataset index count is not a multiple of micro batch size"
        mbs = cfg.micro_batch_size
        for i in range(0, len(idx), mbs):
            self.consumed_samples += mbs * dp
            yield idx[i : i + mbs]


class DataLoader(torch.utils.data.DataLoader):
    def __init__(
        self,
        seed: int,
        consumed_samples: int,
        dataset: BaseDataset,
        topology: Any,
        num_workers: int = 0,
        pin_memory: bool = True,
        prefetch_factor: Optional[int] = None,
        shuffle: bool = True,
    ) -> None:
        self.seed = seed
        self.consumed_samples = consumed_samples
        self.dataset = dataset
        self.topology = topology
        assert len(dataset) >= topology.config.micro_batch_size, (
            f"cannot instantiate data loader with micro_batch_size {topology.config.micro_batch_size} "
            f"because dataset has only length {len(dataset)}"
        )
        sampler = RandomSampler(dataset, seed, consumed_samples, topology, shuffle)
        self.dataloader = torch.utils.data.DataLoader(
            dataset=dataset,
            batch_sampler=sampler,
            num_workers=num_workers,
            collate_fn=dataset.collate,
            pin_memory=pin_memory and torch.cuda.is_available(),
            prefetch_factor=prefetch_factor if num_workers > 0 else None,
        )
        self.iterator = self._iterate()

    def _iterate(self) -> Generator[Any, None, None]:
        while True:
            # torch's loader iterator draws a base seed from the global CPU generator; keep that draw
            # from shifting the training RNG stream so a resumed run replays dropout masks exactly
            state = torch.get_rng_state()
            it = iter(self.dataloader)
            torch.set_rng_state(state)
            for item in it:
                yield item

    def __next__(self) -> Any:
        return next(self.iterator)

    def __iter__(self) -> Any:
        return self
