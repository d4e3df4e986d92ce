"""InferenceModule: layer split over a device list, HiddenStateRecorder, and consistency with a
ParallelModule checkpoint (reference ``tests/core/test_nn/test_inference_module.py:54-198``).

The device lists run on CPU here (``("cpu",)``, ``("cpu", "cpu")``) and on the MI355X box
(``(0,)``, ``(0, 0)``, ``("cpu", 0)`` — a single GPU stands in for the reference's (0, 1)).
"""
from __future__ import annotations

from pathlib import Path

import pytest
import torch

from scaling_amd.core import BaseLayerIO, Topology, TopologyConfig
from scaling_amd.core.nn.parallel_module import ParallelModule
from scaling_amd.core.nn.parallel_module.inference_module import InferenceModule, RecorderSetting
from tests.minimal_model import MinimalBatch, layer_specs

GPU = pytest.mark.gpu
DEVICE_SETS = [
    pytest.param(("cpu",), id="cpu"),
    pytest.param(("cpu", "cpu"), id="cpu-cpu"),
    pytest.param((0,), id="gpu0", marks=GPU),
    pytest.param((0, 0), id="gpu0-gpu0", marks=GPU),
    pytest.param(("cpu", 0), id="cpu-gpu0", marks=GPU),
]


def _dev(d) -> torch.device:
    return torch.device(d) if isinstance(d, str) else torch.device("cuda", d)


def _batch() -> MinimalBatch:
    return MinimalBatch(inputs=torch.tensor([[0, 1, 5]], dtype=torch.long), targets=torch.tensor([[0, 1, 5]]))


@pytest.mark.parametrize("devices", DEVICE_SETS)
@pytest.mark.parametrize("weight_tying", [True, False])
def test_inference_module_init_and_forward_pass(devices, weight_tying):
    m = InferenceModule(layer_specs=layer_specs(weight_tying), devices=devices)
    assert len(m._layers) == 4
    per_stage = 4 // len(devices)
    for k, layer in enumerate(m._layers):
        want = _dev(devices[k // per_stage])
        assert m._layer_devices[k] == want
        for p in layer.parameters():
            assert p.device == want
    out = m(_batch())
    assert out.activations.device == _dev(devices[-1])
    assert out.activations.shape[-1] == (16 if weight_tying else 8)


@pytest.mark.parametrize("devices", DEVICE_SETS)
@pytest.mark.parametrize("requested_layers", [[], [0, 1, 2, 3], [1, 3], [-1]])
@pytest.mark.parametrize("include,exclude", [(None, None), ([""], None), (None, ["", "norm"])])
def test_hidden_state_extraction(devices, requested_layers, include, exclude):
    m = InferenceModule(layer_specs=layer_specs(False), devices=devices)
    settings = {k: RecorderSetting(include_modules=include, exclude_modules=exclude) for k in requested_layers}
    _, hidden = m.forward_with_hidden_state_recorder(_batch(), recorder_settings_per_layer=settings)
    assert set(hidden.keys()) == set(requested_layers)
    submodule = {0: "embedding", 1: "linear", 2: "linear", 3: "norm", -1: "norm"}
    for li, rec in hidden.items():
        if include is None and exclude is None:
            assert len(rec) == 0
        elif include is not None:
            assert set(rec.keys()) == set(include)
        else:
            assert set(rec.keys()) == ({submodule[li]} - {"norm"})
        for k, v in rec.items():
            assert isinstance(v, BaseLayerIO if k == "" else torch.Tensor)


@pytest.mark.parametrize("devices", DEVICE_SETS)
def test_hidden_state_settings_differ_per_layer(devices):
    m = InferenceModule(layer_specs=layer_specs(False), devices=devices)
    settings = {1: RecorderSetting(include_modules=[""]), 2: RecorderSetting(include_modules=["linear"])}
    out, hidden = m.forward_with_hidden_state_recorder(_batch(), recorder_settings_per_layer=settings)
    assert set(hidden[1].keys()) == {""} and set(hidden[2].keys()) == {"linear"}
    # the recorded output of layer 2's linear is the row-parallel projection feeding the final norm
    with torch.no_grad():
        again = m._layers[3].norm(hidden[2]["linear"].to(m._layer_devices[3]))
    torch.testing.assert_close(again, out.activations)
    # hooks are removed after the recorder exits
    assert all(len(mod._forward_hooks) == 0 for layer in m._layers for mod in layer.modules())


@pytest.mark.parametrize("devices", DEVICE_SETS)
@pytest.mark.parametrize("weight_tying", [True, False])
def test_consistency_with_parallel_module(tmp_path: Path, devices, weight_tying):
    gpu = any(not isinstance(d, str) for d in devices)
    topo = Topology(TopologyConfig(global_rank=0, world_size=1, local_slot=0, model_parallel_size=1,
                                   pipe_parallel_size=1, data_parallel_size=1, micro_batch_size=1,
                                   gradient_accumulation_steps=1, backend=None if gpu else "gloo"))
    topo.initialize_device()
    torch.manual_seed(0)
    pm = ParallelModule(layer_specs=layer_specs(weight_tying, topology=topo), topology=topo)
    pm.eval()
    (tmp_path / "ck").mkdir()
    pm.save_checkpoint(tmp_path / "ck")
    x = _batch()
    x.to_(topo.device)
    with torch.no_grad():
        ref = pm(x).activations.cpu()
    m = InferenceModule(layer_specs=layer_specs(weight_tying), devices=devices)
    m.load_checkpoint(tmp_path / "ck")
    out = m(_batch()).activations.cpu()
    torch.testing.assert_close(out, ref)
