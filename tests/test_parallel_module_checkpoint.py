"""ParallelModule checkpoint loading (reference ``tests/core/test_nn/test_parallel_module.py``): a weight set spread
over several directories loads as one; a missing directory is an error; ``ignore_keys_in_checkpoint`` keeps the
fresh initialisation of exactly the ignored parameters and loads everything else bit for bit."""
from __future__ import annotations

from pathlib import Path

import pytest
import torch

from scaling_amd.core import ParallelModule, Topology, TopologyConfig
from tests.minimal_model import layer_specs

pytestmark = pytest.mark.cpu


def _model(seed: int) -> ParallelModule:
    topo = Topology(TopologyConfig(global_rank=0, world_size=1, local_slot=0, model_parallel_size=1,
                                   pipe_parallel_size=1, data_parallel_size=1, micro_batch_size=1,
                                   gradient_accumulation_steps=1, backend="gloo"))
    topo.initialize_device()
    torch.manual_seed(seed)
    return ParallelModule(layer_specs=layer_specs(False, topology=topo), topology=topo)


def _state(m: ParallelModule) -> dict[str, torch.Tensor]:
    return {n: p.detach().clone() for n, p in m.named_parameters()}


def test_load_from_multiple_dirs(tmp_path: Path):
    src = _model(0)
    src.save_checkpoint(tmp_path)
    moved = tmp_path / "layer_3"
    moved.mkdir()
    f = next(tmp_path.glob("model_state_layer_3_*.pt"))
    f.rename(moved / f.name)
    dst = _model(1)
    dst.load_checkpoint([tmp_path, moved], allowed_missing_keys_in_checkpoint=[],
                        allowed_unexpected_keys_in_checkpoint=[], ignore_keys_in_checkpoint=None)
    for (n, a), b in zip(_state(src).items(), _state(dst).values()):
        assert torch.equal(a, b), n
    with pytest.raises(Exception):  # the moved layer is missing when only the top directory is given
        _model(2).load_checkpoint(tmp_path)


def test_load_from_missing_dir_raises(tmp_path: Path):
    src = _model(0)
    src.save_checkpoint(tmp_path)
    with pytest.raises(RuntimeError):
        _model(1).load_checkpoint([tmp_path, tmp_path / "wrong_path"])


def test_ignore_keys_keep_initialisation(tmp_path: Path):
    src = _model(0)
    src.save_checkpoint(tmp_path)
    dst = _model(1)
    fresh = _state(dst)
    dst.load_checkpoint(tmp_path, ignore_keys_in_checkpoint=["embedding.weight"])
    loaded, orig = _state(dst), _state(src)
    for n in orig:
        if n.endswith("embedding.weight"):
            assert torch.equal(loaded[n], fresh[n]) and not torch.equal(loaded[n], orig[n])
        else:
            assert torch.equal(loaded[n], orig[n]), n
