"""MNIST for the MLP example.  Reads the standard idx files when present under ``root``
(``train-images-idx3-ubyte`` / ``train-labels-idx1-ubyte`` / ``t10k-*``, optionally ``.gz``); with no
files (no network on the build machines) a fixed synthetic MNIST-shaped set is used: 28x28 inputs
whose labels come from a random linear teacher, so the model can still learn."""
from __future__ import annotations

import gzip
import struct
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from scaling_amd.core import BaseDataset, BaseDatasetBatch, BaseDatasetItem, Topology, broadcast_data


def _read_idx(path: Path) -> Optional[np.ndarray]:
    for p in (path, Path(str(path) + ".gz")):
        if p.is_file():
            raw = gzip.open(p, "rb").read() if p.suffix == ".gz" else p.read_bytes()
            _, _, dt, nd = struct.unpack(">HBBB", raw[:4])
            dims = struct.unpack(">" + "I" * nd, raw[4 : 4 + 4 * nd])
            return np.frombuffer(raw, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)
    return None


class MNISTDatasetItem(BaseDatasetItem):
    def __init__(self, input_: np.ndarray, target: int):
        self.input = torch.tensor(input_, dtype=torch.float16)
        self.target = torch.tensor(target, dtype=torch.float16)


class MNISTDatasetBatch(BaseDatasetBatch):
    def __init__(self, inputs: Optional[torch.Tensor] = None, targets: Optional[torch.Tensor] = None):
        self.inputs = inputs
        self.targets = targets

    def only_inputs(self) -> "MNISTDatasetBatch":
        return MNISTDatasetBatch(inputs=self.inputs)

    def only_targets(self) -> "MNISTDatasetBatch":
        return MNISTDatasetBatch(targets=self.targets)


class MNISTDataset(BaseDataset[MNISTDatasetItem, MNISTDatasetBatch, MNISTDatasetBatch]):
    def __init__(self, root: Path = Path(".data"), train: bool = True, synthetic_samples: int = 8192):
        split = "train" if train else "t10k"
        images = _read_idx(Path(root) / f"{split}-images-idx3-ubyte")
        labels = _read_idx(Path(root) / f"{split}-labels-idx1-ubyte")
        if images is not None and labels is not None:
            self.x = (images.astype(np.float32) / 255.0 - 0.5) / 0.5
            self.y = labels.astype(np.int64)
            self.synthetic = False
        else:
            rng = np.random.RandomState(0 if train else 1)
            n = synthetic_samples if train else max(synthetic_samples // 8, 256)
            self.x = rng.randn(n, 28, 28).astype(np.float32)
            teacher = np.random.RandomState(1234).randn(28 * 28, 10).astype(np.float32)
            self.y = (self.x.reshape(n, -1) @ teacher).argmax(-1).astype(np.int64)
            self.synthetic = True
        super().__init__(seed=0)

    def __len__(self) -> int:
        return len(self.y)

    def __getitem__(self, index: int) -> MNISTDatasetItem:
        return MNISTDatasetItem(input_=self.x[index][None], target=int(self.y[index]))

    def ident(self) -> str:
        return "MNIST" + ("-synthetic" if self.synthetic else "")

    def set_seed(self, seed: int, shuffle: bool = True) -> None:
        return

    def collate(self, batch: list[MNISTDatasetItem]) -> MNISTDatasetBatch:
        return MNISTDatasetBatch(inputs=torch.stack([b.input for b in batch]), targets=torch.stack([b.target for b in batch]))

    @staticmethod
    def sync_batch_to_model_parallel(topology: Topology, batch: Optional[MNISTDatasetBatch]) -> MNISTDatasetBatch:
        if topology.model_parallel_rank == 0:
            assert batch is not None
            tensors: list[Optional[torch.Tensor]] = [batch.inputs, batch.targets]
        else:
            assert batch is None
            tensors = [None, None]
        out = broadcast_data(tensors=tensors, dtype=torch.float16, topology=topology)
        return MNISTDatasetBatch(inputs=out[0], targets=out[1])
