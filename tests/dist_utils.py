"""Multi-process helpers for CPU (gloo) tests: spawn `world_size` ranks on 127.0.0.1, collect results."""
from __future__ import annotations

import os
import traceback
from typing import Any, Callable

import torch.multiprocessing as mp


def free_port() -> int:
    from scaling_amd.core.utils.port import find_free_port

    return find_free_port()


def _entry(rank: int, world_size: int, port: int, fn: Callable, kwargs: dict, q: Any) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world_size),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world_size))
    try:
        q.put((rank, fn(**kwargs), None))
    except Exception:  # noqa: BLE001 - surfaced in the parent
        q.put((rank, None, traceback.format_exc()))


def run_distributed(fn: Callable, world_size: int, timeout: float = 300.0, **kwargs: Any) -> dict[int, Any]:
    """Runs fn(**kwargs) on every rank; returns {rank: result}; raises if any rank failed."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world_size, port, fn, kwargs, q)) for r in range(world_size)]
    for p in procs:
        p.start()
    out: dict[int, Any] = {}
    errors = []
    for _ in range(world_size):
        rank, res, err = q.get()
        if err is not None:
            errors.append(f"rank {rank}:\n{err}")
        out[rank] = res
    for p in procs:
        p.join(timeout=timeout)
        if p.is_alive():
            p.kill()
    if errors:
        raise RuntimeError("\n".join(errors))
    return out


def make_topology(model_parallel_size: int = 1, pipe_parallel_size: int = 1, micro_batch_size: int = 2,
                  gradient_accumulation_steps: int = 1, **extra: Any):
    """Topology for the calling rank (env from run_distributed), distributed initialised on gloo."""
    from scaling_amd.core import Topology, TopologyConfig

    world = int(os.environ["WORLD_SIZE"])
    cfg = TopologyConfig(global_rank=int(os.environ["RANK"]), world_size=world, local_slot=int(os.environ["LOCAL_RANK"]),
                         model_parallel_size=model_parallel_size, pipe_parallel_size=pipe_parallel_size,
                         data_parallel_size=world // (model_parallel_size * pipe_parallel_size),
                         micro_batch_size=micro_batch_size, gradient_accumulation_steps=gradient_accumulation_steps,
                         **extra)
    topo = Topology(config=cfg)
    topo.initialize_distributed(master_addr="127.0.0.1", master_port=os.environ["MASTER_PORT"],
                                torch_distributed_timeout_minutes=2)
    return topo
