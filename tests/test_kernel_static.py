"""Static (compile-only, no GPU) checks of the HIP kernels' generated gfx950 code."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")
def test_attention_barriers_retire_lds_dma():
    """Every barrier of the attention loops that hands LDS-DMA-staged tiles to other waves is preceded, in program
    order, by s_waitcnt vmcnt(0) with no DMA issue in between (the round-5 race: a wave read a slower peer's piece of
    the next tile before it landed).  tools/dma_barrier_check.py compiles flash_fwd.hip / flash_bwd.hip and walks the
    assembly."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dma_barrier_check.py")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
