"""Multi-node job runner (reference ``runner/runner.py``): resource pool from hostsfile / hosts / local
GPUs, env export (NCCL_*/RCCL_*/HSA_*/HIP_*/PYTHON*/UCX_*), pdsh fan-out (skipped for localhost-only
pools), optional docker with ROCm device flags."""
from __future__ import annotations

import os
import re
import subprocess
import sys
from pathlib import Path
from typing import Any, Optional

from ..utils.debug_env import debug_env
from .launch_config import encode_base64
from .runner_config import RunnerConfig, RunnerType

EXPORT_ENVS = ["NCCL", "RCCL", "HSA", "HIP", "ROCR", "AMD", "PYTHON", "MV2", "UCX", "TORCH", "OMP"]


def parse_host(line: str, default_gpu_count: int) -> tuple[str, list[int]]:
    """'host slots=0,1,3' | 'host slots=4' | 'host' -> (host, slots)."""
    line = line.strip()
    m = re.match(r"^(\S+)(?:\s+slots=(\S+))?$", line)
    if m is None:
        raise ValueError(f"bad host line: {line}")
    host, slots = m.group(1), m.group(2)
    if slots is None:
        return host, list(range(default_gpu_count))
    if "," in slots:
        return host, [int(s) for s in slots.split(",") if s]
    n = int(slots)
    return host, list(range(n))


def hosts_str_to_resource_pool(hosts: list[str], default_gpu_count: int) -> dict[str, list[int]]:
    pool: dict[str, list[int]] = {}
    for h in hosts:
        if not h.strip() or h.strip().startswith("#"):
            continue
        name, slots = parse_host(h, default_gpu_count)
        pool[name] = slots
    return pool


def get_resource_pool(config: RunnerConfig) -> dict[str, list[int]]:
    if config.hostsfile is not None:
        return hosts_str_to_resource_pool(Path(config.hostsfile).read_text().splitlines(), config.default_gpu_count)
    if config.hosts is not None:
        return hosts_str_to_resource_pool(config.hosts, config.default_gpu_count)
    try:
        import torch

        n = torch.cuda.device_count() or config.default_gpu_count
    except Exception:  # noqa: BLE001
        n = config.default_gpu_count
    return {"localhost": list(range(n))}


def _exports(config: Optional[RunnerConfig] = None) -> dict[str, str]:
    env = {k: v for k, v in os.environ.items() if any(k.startswith(p) for p in EXPORT_ENVS)}
    if config is not None:
        env.update(debug_env(config.debug_collectives, config.debug_hip_launch_blocking, config.debug_single_stream))
    extra = Path.home() / ".deepspeed_env"
    if extra.is_file():
        for line in extra.read_text().splitlines():
            if "=" in line:
                k, v = line.split("=", 1)
                env[k.strip()] = v.strip()
    return env


class PDSHRunner:
    def __init__(self, config: RunnerConfig, pool: dict[str, list[int]], master_addr: str):
        self.config, self.pool, self.master_addr = config, pool, master_addr

    def get_cmd(self, payload: Optional[dict[str, Any]] = None) -> list[str]:
        launch = [
            sys.executable, "-u", "-m", "scaling_amd.core.runner.launch",
            f"--resource_pool={encode_base64(self.pool)}", f"--master_addr={self.master_addr}",
            f"--master_port={self.config.master_port}",
        ]
        script = [str(self.config.script)] + (["--payload", encode_base64(payload)] if payload is not None else [])
        local_only = all(h in ("localhost", "127.0.0.1") for h in self.pool)
        if local_only:
            return launch + ["--node_rank=0"] + script
        exports = " ".join(f"export {k}={v};" for k, v in _exports(self.config).items())
        inner = " ".join(launch + ["--node_rank=%n"] + script)
        if self.config.runner_type == RunnerType.PDSH_DOCKER:
            d = self.config.docker_config
            mounts = " ".join(f"-v {a}:{b}" for a, b in (d.docker_mounts or []))
            sudo = "sudo " if d.docker_sudo else ""
            inner = (f"{sudo}docker run --rm --network=host --ipc=host --device=/dev/kfd --device=/dev/dri "
                     f"--group-add video --security-opt seccomp=unconfined {mounts} {d.docker_container} "
                     f"bash -c '{inner}'")
        return ["pdsh", "-S", "-f", "1024", "-w", ",".join(self.pool.keys()), f"cd {os.getcwd()}; {exports} {inner}"]


def runner_main(config: RunnerConfig, payload: Optional[dict[str, Any]] = None) -> int:
    pool = get_resource_pool(config)
    hosts = list(pool.keys())
    if config.master_addr is not None:
        master = config.master_addr
    elif hosts[0] in ("localhost", "127.0.0.1"):
        master = "127.0.0.1"
    else:
        out = subprocess.check_output(["ssh", hosts[0], "hostname -I"], text=True)
        master = out.split()[0]
    cmd = PDSHRunner(config, pool, master).get_cmd(payload)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(debug_env(config.debug_collectives, config.debug_hip_launch_blocking, config.debug_single_stream))
    proc = subprocess.Popen(cmd, env=env)
    rc = proc.wait()
    if rc != 0:  # the failing rank already printed its error; propagate the code quietly
        sys.exit(rc)
    return rc
