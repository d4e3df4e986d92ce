"""Environment switches for deterministic runs and for debugging collectives / HIP launches
(SURVEY §5.2 MI355X plan).  The runner exports them to every rank; ``apply`` sets them in-process
before the first HIP / RCCL call."""
from __future__ import annotations

import os
from typing import Mapping

# RCCL honours the NCCL_* names; TORCH_* are torch.distributed's own switches
COLLECTIVE_DEBUG_ENV: Mapping[str, str] = {
    "NCCL_DEBUG": "INFO",
    "NCCL_DEBUG_SUBSYS": "INIT,COLL,P2P",
    "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",
    "TORCH_NCCL_DUMP_ON_TIMEOUT": "1",
    "TORCH_DISTRIBUTED_DEBUG": "DETAIL",
}

# every kernel launch synchronous and serialized, so a fault is reported at the launch that caused it
HIP_LAUNCH_DEBUG_ENV: Mapping[str, str] = {
    "HIP_LAUNCH_BLOCKING": "1",
    "AMD_SERIALIZE_KERNEL": "3",
    "AMD_SERIALIZE_COPY": "3",
}

# library-side determinism: rocBLAS without atomics, no online GEMM re-tuning (TunableOp only reads its
# fixed solution table, so every run picks the same kernels); the package's own HIP kernels reduce in a
# fixed order (no float atomics)
DETERMINISTIC_ENV: Mapping[str, str] = {
    "CUBLAS_WORKSPACE_CONFIG": ":4096:8",
    "ROCBLAS_DEFAULT_ATOMICS_MODE": "0",
    "PYTORCH_TUNABLEOP_TUNING": "0",
}


# race check: every side stream (DP communication, overlapped optimizer step, weight-gradient stream) folds onto
# the compute stream, so the run is the serialized schedule of the same kernels.  A run whose parameters differ
# from its SCALING_AMD_SINGLE_STREAM=1 twin has a missing stream / event dependency (tests/test_gpu_rehearsal.py).
SINGLE_STREAM_ENV: Mapping[str, str] = {"SCALING_AMD_SINGLE_STREAM": "1"}


# race check with a late communication stream: SCALING_AMD_COMM_DELAY_US=<us> enqueues a busy-wait kernel of that
# length on the DP communication stream in front of every gradient reduce-scatter and parameter all-gather, so a
# consumer that forgot to wait for the stream reads stale data with near certainty instead of by timing luck.
# Results must stay bit-identical to the undelayed run (tests/test_gpu_rehearsal.py).
def comm_delay_us() -> int:
    try:
        return max(0, int(os.environ.get("SCALING_AMD_COMM_DELAY_US", "0") or 0))
    except ValueError:
        return 0


SIDE_STREAM_FEATURES = ("dp_comm", "opt_step", "wgrad", "tp_comm")


def side_streams_enabled(feature: str = "") -> bool:
    """Whether side-stream ``feature`` runs on its own stream.  ``SCALING_AMD_SINGLE_STREAM`` = 1 folds every side
    stream onto the compute stream; a comma-separated subset of ``SIDE_STREAM_FEATURES`` folds only those (the race
    check bisects a multi- vs single-stream difference this way):
      dp_comm   the data-parallel gradient reduce-scatter / parameter all-gather stream (optimizer)
      opt_step  the overlapped optimizer update (its own stream when there is no DP stream)
      wgrad     the weight-gradient GEMM stream (SCALING_AMD_WGRAD_STREAM=1)
      tp_comm   the tensor-parallel collective stream of the chunked row-parallel GEMMs"""
    v = os.environ.get("SCALING_AMD_SINGLE_STREAM", "0").strip()
    if v in ("", "0"):
        return True
    if v in ("1", "all"):
        return False
    folded = {f.strip() for f in v.split(",")}
    unknown = folded - set(SIDE_STREAM_FEATURES)
    assert not unknown, f"SCALING_AMD_SINGLE_STREAM: unknown features {sorted(unknown)} (known: {SIDE_STREAM_FEATURES})"
    return feature not in folded


def debug_env(collectives: bool = False, hip_launch_blocking: bool = False, single_stream: bool = False
              ) -> dict[str, str]:
    env: dict[str, str] = {}
    if collectives:
        env.update(COLLECTIVE_DEBUG_ENV)
    if hip_launch_blocking:
        env.update(HIP_LAUNCH_DEBUG_ENV)
    if single_stream:
        env.update(SINGLE_STREAM_ENV)
    return env


def apply(env: Mapping[str, str], override: bool = False) -> None:
    for k, v in env.items():
        if override or k not in os.environ:
            os.environ[k] = v
