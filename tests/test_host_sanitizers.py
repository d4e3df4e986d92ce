"""Host-code sanitizers: the native data-index builders (csrc/data/data_index_core.h) are
compiled with AddressSanitizer + UndefinedBehaviorSanitizer into a standalone harness and run.  GPU
sanitizers are not available on this pool; this covers the C++ host library."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_data_index_asan_ubsan(tmp_path):
    exe = tmp_path / "data_index_asan"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", str(ROOT / "csrc" / "tests" / "data_index_asan.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "harness ok" in r.stdout
