from .launch_config import LaunchConfig, decode_base64, encode_base64
from .runner import runner_main
from .runner_config import RunnerConfig, RunnerDockerConfig, RunnerType

__all__ = ["LaunchConfig", "RunnerConfig", "RunnerDockerConfig", "RunnerType", "decode_base64", "encode_base64", "runner_main"]
