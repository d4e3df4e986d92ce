"""Runner / launcher end to end on localhost (reference: tests/core/test_runner/test_runner.py): the pdsh
runner skips pdsh for a localhost-only pool and the per-node launcher spawns one process per slot with the
right RANK / WORLD_SIZE / LOCAL_SLOT; a failing rank makes the launcher kill its siblings (fail fast)."""
import json
import time
from pathlib import Path

import pytest

pytestmark = pytest.mark.cpu
SCRIPT = Path(__file__).resolve().parent / "files" / "runner_script.py"


def _config(tmp: Path, hosts, use_hostsfile: bool):
    from scaling_amd.core import RunnerConfig

    hostsfile = None
    if use_hostsfile:
        hostsfile = tmp / "hostfile"
        hostsfile.write_text("".join(f"{h}\n" for h in hosts))
    return RunnerConfig.from_dict({
        "runner_type": "pdsh", "hostsfile": str(hostsfile) if hostsfile else None,
        "hosts": None if use_hostsfile else hosts, "master_port": 29731, "master_addr": None, "script": str(SCRIPT),
        "default_gpu_count": 8,
        "docker_config": {"docker_container": "container_name", "docker_sudo": False, "docker_mounts": None},
    })


@pytest.mark.parametrize("hosts,world", [(["localhost"], 8), (["localhost slots=8"], 8), (["localhost slots=0,"], 1),
                                         (["localhost slots=0,1,2"], 3)])
@pytest.mark.parametrize("use_hostsfile", [True, False])
def test_runner_spawns_one_process_per_slot(tmp_path, hosts, world, use_hostsfile):
    from scaling_amd.core import runner_main

    rc = runner_main(config=_config(tmp_path, hosts, use_hostsfile), payload={"cache_dir": str(tmp_path)})
    assert rc == 0
    outs = sorted(tmp_path.glob("process_*.json"))
    assert len(outs) == world
    cfgs = [json.loads(o.read_text()) for o in outs]
    assert sorted(c["global_rank"] for c in cfgs) == list(range(world))
    assert all(c["world_size"] == world for c in cfgs)


def test_launcher_fails_fast(tmp_path):
    from scaling_amd.core import runner_main

    t0 = time.time()
    with pytest.raises(SystemExit) as e:
        runner_main(config=_config(tmp_path, ["localhost slots=0,1,2"], False),
                    payload={"cache_dir": str(tmp_path), "fail_rank": 1})
    assert e.value.code != 0
    assert time.time() - t0 < 45, "siblings were not killed after the failing rank exited"


def test_runner_config_legacy_hostfile_alias(tmp_path):
    from scaling_amd.core import RunnerConfig

    hf = tmp_path / "hostfile"
    hf.write_text("localhost")
    c = RunnerConfig.from_dict({"hostfile": str(hf), "script": str(SCRIPT)})
    assert str(c.hostsfile) == str(hf)


def test_runner_debug_and_determinism_env(monkeypatch):
    from scaling_amd.core.runner.runner import PDSHRunner, _exports
    from scaling_amd.core.runner.runner_config import RunnerConfig
    from scaling_amd.core.utils import debug_env

    cfg = RunnerConfig(hosts=["worker-0 slots=0,1", "worker-1 slots=0,1"], debug_collectives=True,
                       debug_hip_launch_blocking=True, script="train.py")
    env = _exports(cfg)
    assert env["NCCL_DEBUG"] == "INFO" and env["HIP_LAUNCH_BLOCKING"] == "1" and env["AMD_SERIALIZE_KERNEL"] == "3"
    cmd = PDSHRunner(cfg, {"worker-0": [0, 1], "worker-1": [0, 1]}, "10.0.0.1").get_cmd()
    assert "export NCCL_DEBUG=INFO;" in cmd[-1] and "export HIP_LAUNCH_BLOCKING=1;" in cmd[-1]
    assert "NCCL_DEBUG" not in _exports(RunnerConfig(hosts=["localhost"]))
    for k in debug_env.DETERMINISTIC_ENV:  # registered with monkeypatch: restored after the test
        monkeypatch.delenv(k, raising=False)
    debug_env.apply(debug_env.DETERMINISTIC_ENV)
    import os

    assert os.environ["ROCBLAS_DEFAULT_ATOMICS_MODE"] == "0" and os.environ["PYTORCH_TUNABLEOP_TUNING"] == "0"


def test_single_stream_race_check_switch(monkeypatch):
    from scaling_amd.core.utils.debug_env import debug_env, side_streams_enabled

    monkeypatch.delenv("SCALING_AMD_SINGLE_STREAM", raising=False)
    assert side_streams_enabled()
    monkeypatch.setenv("SCALING_AMD_SINGLE_STREAM", "1")
    assert not side_streams_enabled()
    assert debug_env(single_stream=True) == {"SCALING_AMD_SINGLE_STREAM": "1"}
