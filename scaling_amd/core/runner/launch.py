"""Per-node launcher: one process per local GPU slot, fail-fast (reference ``runner/launch.py``).

Spawns ``python -u SCRIPT --payload B64`` per slot with MASTER_ADDR/PORT, WORLD_SIZE, RANK,
LOCAL_SLOT (and LOCAL_RANK) set, plus ``HIP_VISIBLE_DEVICES`` untouched (every rank sees all GPUs and
binds ``local_slot``); polls children, kills all on the first failure, forwards SIGINT/SIGTERM.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from argparse import ArgumentParser, Namespace
from typing import Any

from .launch_config import decode_base64


def parse_args(argv: list[str] | None = None) -> Namespace:
    p = ArgumentParser(description="process launch")
    p.add_argument("--node_rank", type=int, default=0)
    p.add_argument("--master_addr", default="127.0.0.1", type=str)
    p.add_argument("--master_port", default=29500, type=int)
    p.add_argument("--resource_pool", required=True, type=str, help="base64 encoded {host: [slots]}")
    p.add_argument("script", type=str)
    p.add_argument("--payload", type=str, default=None)
    return p.parse_args(argv)


def main(argv: list[str] | None = None) -> int:
    args = parse_args(argv)
    pool: dict[str, list[int]] = decode_base64(args.resource_pool)
    hosts = list(pool.keys())
    host = hosts[args.node_rank]
    world = sum(len(v) for v in pool.values())
    first_rank = sum(len(pool[h]) for h in hosts[: args.node_rank])
    if not pool[host]:
        print(f"[launch] no slots for host {host} in the resource pool (e.g. 'host slots=8')", file=sys.stderr)
        return 2
    procs: list[subprocess.Popen[Any]] = []
    for i, slot in enumerate(pool[host]):
        env = dict(os.environ)
        env.update(MASTER_ADDR=args.master_addr, MASTER_PORT=str(args.master_port), WORLD_SIZE=str(world),
                   RANK=str(first_rank + i), LOCAL_SLOT=str(slot), LOCAL_RANK=str(slot))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        cmd = [sys.executable, "-u", args.script] + (["--payload", args.payload] if args.payload else [])
        procs.append(subprocess.Popen(cmd, env=env))

    def kill_all(*_: Any) -> None:
        for p in procs:
            if p.poll() is None:
                p.kill()

    def on_signal(signum: int, _frame: Any) -> None:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        kill_all()
        sys.exit(1)

    signal.signal(signal.SIGINT, on_signal)
    signal.signal(signal.SIGTERM, on_signal)
    alive = list(procs)
    while alive:
        for p in list(alive):
            rc = p.poll()
            if rc is None:
                continue
            alive.remove(p)
            if rc != 0:
                kill_all()
                return rc
        time.sleep(1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
