"""hipBLASLt solution selection for the framework's GEMM shapes via PyTorch TunableOp.

hipBLASLt's default heuristic picks measurably slower solutions for some of the transformer's
layouts on gfx950 (see ``profiles/``).  The shipped table ``scaling_amd/tuning/gemm_gfx950.csv`` was
produced on MI355X by ``tune`` mode (every solution benchmarked with a rotating buffer larger than
the 256 MB MALL so timings reflect cold caches).  ``use`` mode loads it with tuning disabled; any
shape not in the table falls back to the library heuristic.  ``SCALING_AMD_GEMM_TABLE`` points ``use`` mode at another
table (A/B of a re-tuned one); ``SCALING_AMD_GEMM_RETUNE=1`` makes ``tune`` mode start from an empty table instead of
extending the shipped one.  The file carries TunableOp's validator
lines (torch / HIP / hipBLASLt versions): a mismatching software stack rejects it as a whole.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from pathlib import Path
from typing import Optional

import torch

TUNED_FILE = Path(__file__).resolve().parent.parent / "tuning" / "gemm_gfx950.csv"


def enable_tuned_gemms(mode: Optional[str] = None, out_path: Optional[str] = None, rank: int = 0) -> str:
    """mode: "use" (default if the table exists), "tune" (benchmark unseen shapes, write ``out_path``), "off"."""
    mode = mode or os.environ.get("SCALING_AMD_GEMM_TUNING", "use")
    if mode == "off" or not torch.cuda.is_available():
        return "off"
    tun = torch.cuda.tunable
    if mode == "tune":
        path = out_path or str(Path(tempfile.gettempdir()) / f"sa_gemm_tuning_{rank}.csv")
        if TUNED_FILE.is_file() and not Path(path).exists() and os.environ.get("SCALING_AMD_GEMM_RETUNE") != "1":
            shutil.copy(TUNED_FILE, path)  # extend the shipped table
        tun.set_filename(path, insert_device_ordinal=False)
        tun.set_rotating_buffer_size(512)
        tun.set_max_tuning_duration(150)
        tun.set_max_tuning_iterations(int(os.environ.get("SCALING_AMD_GEMM_TUNE_ITERS", "60")))
        tun.enable(True)
        tun.tuning_enable(True)
        return "tune"
    table = Path(os.environ.get("SCALING_AMD_GEMM_TABLE", "") or TUNED_FILE)
    if not table.is_file():
        return "off"
    # private per-rank copy: TunableOp rewrites its file at exit
    path = str(Path(tempfile.gettempdir()) / f"sa_gemm_tuned_{os.getpid()}.csv")
    shutil.copy(table, path)
    tun.set_filename(path, insert_device_ordinal=False)
    tun.enable(True)
    tun.tuning_enable(False)
    return "use"


def write_tuning_file() -> None:
    if torch.cuda.is_available() and torch.cuda.tunable.is_enabled():
        torch.cuda.tunable.write_file() if hasattr(torch.cuda.tunable, "write_file") else None
