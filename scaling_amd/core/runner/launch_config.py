"""Per-process launch configuration from env + ``--payload`` (reference ``runner/launch_config.py``).

Accepts the framework launcher's env (``LOCAL_SLOT``) and torchrun's (``LOCAL_RANK``)."""
from __future__ import annotations

import base64
import json
import os
from argparse import REMAINDER, ArgumentParser
from pathlib import Path
from typing import Any, Optional

from pydantic import Field

from ..config import BaseConfig


def encode_base64(d: dict[Any, Any]) -> str:
    return base64.urlsafe_b64encode(json.dumps(d).encode("utf-8")).decode("utf-8")


def decode_base64(s: str) -> dict[Any, Any]:
    return json.loads(base64.urlsafe_b64decode(s))


class LaunchConfig(BaseConfig):
    master_port: int = Field(description="torch.distributed rendezvous port")
    master_addr: str = Field(description="IP address of the master node")
    world_size: int = Field(description="Total world size of job")
    global_rank: int = Field(description="Global rank of the current process")
    local_slot: int = Field(description="GPU id of the current process")
    payload: Optional[dict[Any, Any]] = Field(None, description="decoded config payload")

    @classmethod
    def from_launcher_args(cls, argv: Optional[list[str]] = None) -> "LaunchConfig":
        parser = ArgumentParser(description="process launch")
        parser.add_argument("--payload", type=str, default=None, help="base64 encoded payload")
        parser.add_argument("remaining_args", nargs=REMAINDER)
        args, _ = parser.parse_known_args(argv)
        return cls(
            master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
            master_port=int(os.environ.get("MASTER_PORT", 29500)),
            world_size=int(os.environ.get("WORLD_SIZE", 1)),
            global_rank=int(os.environ.get("RANK", 0)),
            local_slot=int(os.environ.get("LOCAL_SLOT", os.environ.get("LOCAL_RANK", 0))),
            payload=None if args.payload is None else decode_base64(args.payload),
        )

    def overwrite_config_dict_with_launcher_args(self, config_dict: dict[str, Any]) -> dict[str, Any]:
        config_dict.setdefault("topology", {})
        config_dict["topology"]["world_size"] = self.world_size
        config_dict["topology"]["global_rank"] = self.global_rank
        config_dict["topology"]["local_slot"] = self.local_slot
        prof = config_dict.get("profiler") or {}
        log_dir = (config_dict.get("logger") or {}).get("log_dir")
        if prof.get("profiler_output") is None and log_dir is not None:
            config_dict.setdefault("profiler", {})
            config_dict["profiler"]["profiler_output"] = str(Path(log_dir) / "profile.json")
        return config_dict
