"""``scaling_amd.utils.gemm_tuning``: which TunableOp table is loaded / seeded, on CPU with a stand-in for
``torch.cuda.tunable`` (the real module needs a GPU)."""
from __future__ import annotations

from pathlib import Path

import pytest
import torch

from scaling_amd.utils import gemm_tuning


class _FakeTunable:
    def __init__(self) -> None:
        self.calls: dict = {}

    def __getattr__(self, name):  # set_filename, enable, tuning_enable, set_* knobs
        def rec(*args, **kwargs):
            self.calls[name] = args

        return rec


@pytest.fixture()
def fake(monkeypatch, tmp_path):
    t = _FakeTunable()
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "tunable", t, raising=False)
    monkeypatch.setattr(gemm_tuning.tempfile, "gettempdir", lambda: str(tmp_path))
    for k in ("SCALING_AMD_GEMM_TABLE", "SCALING_AMD_GEMM_RETUNE", "SCALING_AMD_GEMM_TUNE_ITERS", "SCALING_AMD_GEMM_TUNING"):
        monkeypatch.delenv(k, raising=False)
    return t


def test_use_loads_a_private_copy_of_the_shipped_table(fake):
    assert gemm_tuning.enable_tuned_gemms("use") == "use"
    path = Path(fake.calls["set_filename"][0])
    assert path.read_text() == gemm_tuning.TUNED_FILE.read_text()
    assert fake.calls["tuning_enable"] == (False,)


def test_use_takes_the_table_override(fake, monkeypatch, tmp_path):
    other = tmp_path / "other.csv"
    other.write_text("Validator,PT_VERSION,0\n")
    monkeypatch.setenv("SCALING_AMD_GEMM_TABLE", str(other))
    assert gemm_tuning.enable_tuned_gemms("use") == "use"
    assert Path(fake.calls["set_filename"][0]).read_text() == other.read_text()


def test_tune_seeds_from_the_shipped_table_unless_retune(fake, monkeypatch, tmp_path):
    out = tmp_path / "t1.csv"
    assert gemm_tuning.enable_tuned_gemms("tune", str(out)) == "tune"
    assert out.read_text() == gemm_tuning.TUNED_FILE.read_text()
    assert fake.calls["set_max_tuning_iterations"] == (60,)
    monkeypatch.setenv("SCALING_AMD_GEMM_RETUNE", "1")
    monkeypatch.setenv("SCALING_AMD_GEMM_TUNE_ITERS", "10")
    out2 = tmp_path / "t2.csv"
    assert gemm_tuning.enable_tuned_gemms("tune", str(out2)) == "tune"
    assert not out2.exists()  # TunableOp starts from an empty table
    assert fake.calls["set_max_tuning_iterations"] == (10,)


def test_off_touches_nothing(fake):
    assert gemm_tuning.enable_tuned_gemms("off") == "off"
    assert fake.calls == {}
