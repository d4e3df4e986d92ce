from enum import Enum
from pathlib import Path
from typing import Optional

from pydantic import Field

from ..config import BaseConfig


class RunnerType(Enum):
    PDSH = "pdsh"
    PDSH_DOCKER = "pdsh_docker"


class RunnerDockerConfig(BaseConfig):
    docker_container: Optional[str] = Field(None, description="Name of the docker container to be started")
    docker_sudo: bool = Field(False, description="Run docker command with sudo")
    docker_mounts: Optional[list[tuple[str, str]]] = Field(None, description="(host, container) mounts")


class RunnerConfig(BaseConfig, populate_by_name=True):
    runner_type: RunnerType = Field(RunnerType.PDSH, description="Type of the runner to be invoked.")
    hostsfile: Optional[Path] = Field(None, description="MPI-style hostsfile (e.g. 'worker-0 slots=8')", alias="hostfile")
    hosts: Optional[list[str]] = Field(None, description="hosts alternative to hostsfile")
    master_port: int = Field(29500, description="torch.distributed rendezvous port")
    master_addr: Optional[str] = Field(None, description="IP of node 0; inferred via 'hostname -I' if not set")
    script: Optional[Path] = Field(None, description="User script to launch")
    default_gpu_count: int = Field(8, description="GPUs per node if not given in the hosts' slots")
    docker_config: RunnerDockerConfig = Field(RunnerDockerConfig(), description="docker runner configuration")
    use_determined: bool = Field(False, description="use Determined for metric and checkpoint tracking")
    debug_collectives: bool = Field(False, description="export RCCL/torch.distributed debug logging to every rank")
    debug_hip_launch_blocking: bool = Field(
        False, description="export HIP_LAUNCH_BLOCKING / AMD_SERIALIZE_KERNEL: synchronous, serialized kernel launches"
    )
    debug_single_stream: bool = Field(
        False, description="race check: export SCALING_AMD_SINGLE_STREAM (all side-stream work on the compute stream)"
    )
