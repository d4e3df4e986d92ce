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


def test_war_rule_walker_on_synthetic_streams():
    """The WAR walker of tools/dma_barrier_check.py flags an LDS-DMA that can follow a ds_read without an
    lgkmcnt(0) + s_barrier in between -- on the straight path and through a loop's back-edge -- and passes the safe
    forms (so the real kernels' 'ok' is not vacuous)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from dma_barrier_check import war_violations

    dma = "buffer_load_dwordx4 v1, s[4:7], 0 offen lds"
    safe = ["ds_read_b128 v[0:3], v9", "s_waitcnt lgkmcnt(0)", "s_barrier", dma]
    assert war_violations("f", "k", safe) == []
    assert war_violations("f", "k", ["ds_read_b128 v[0:3], v9", "s_barrier", dma])  # read not retired before barrier
    assert war_violations("f", "k", ["ds_read_b128 v[0:3], v9", "s_waitcnt lgkmcnt(0)", dma])  # no barrier
    assert war_violations("f", "k", [dma]) == []  # prologue
    # loop: the DMA at the loop head follows the previous iteration's reads through the back-edge
    loop_bad = [".LBB0_1:", dma, "ds_read_b128 v[0:3], v9", "s_waitcnt lgkmcnt(0)", "s_cbranch_scc1 .LBB0_1"]
    assert war_violations("f", "k", loop_bad)
    loop_ok = [".LBB0_1:", dma, "ds_read_b128 v[0:3], v9", "s_waitcnt lgkmcnt(0)", "s_barrier",
               "s_cbranch_scc1 .LBB0_1"]
    assert war_violations("f", "k", loop_ok) == []
