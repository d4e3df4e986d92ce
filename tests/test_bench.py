"""bench.py contract on CPU (gloo plumbing mode): self-launch of N ranks, one JSON line, fail-fast."""
from __future__ import annotations

import json
import math
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args: list[str], env_extra: dict | None = None, timeout: int = 600) -> subprocess.CompletedProcess:
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out: str) -> list[dict]:
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


TINY = ["--model", "llama_tiny", "--backend", "gloo", "--seq-len", "64", "--micro-batch", "1", "--steps", "2",
        "--warmup", "1"]


@pytest.mark.parametrize("layout", [("4", "2", "2", "2"), ("8", "2", "2", "4"), ("2", "1", "1", "2")])
def test_bench_self_launch_gloo(layout):
    gpus, tp, pp, acc = layout
    r = _run(["--gpus", gpus, "--tp", tp, "--pp", pp, "--grad-acc", acc, *TINY])
    assert r.returncode == 0, r.stderr[-4000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    res = lines[0]
    n = int(gpus)
    dp = n // (int(tp) * int(pp))
    assert res["n_gpus"] == n and res["config"]["world_size_seen"] == n
    assert res["config"]["parallelism"].startswith(f"tp{tp}_pp{pp}_dp{dp}")
    assert res["config"]["global_batch"] == dp * int(acc)
    assert len(res["config"]["per_rank_ms_per_step"]) == n
    assert res["config"]["dp_param_checksum_agree"] is True
    assert res["value"] > 0 and res["steps"] == 2 and res["warmup"] == 1
    assert res["value"] == pytest.approx(res["config"]["global_batch"] * 64 * 2 / (res["ms_per_step"] * 2 / 1000.0))
    assert "NOT headline" in res["config"]["model"]


def test_bench_lora_gloo():
    r = _run(["--gpus", "2", "--lora", "--lora-rank", "8", "--grad-acc", "2", *TINY])
    assert r.returncode == 0, r.stderr[-4000:]
    res = _json_lines(r.stdout)[0]
    assert res["config"]["parallelism"].endswith("_lora") and res["config"]["dp_param_checksum_agree"]


def test_bench_launcher_fail_fast():
    t0 = time.time()
    r = _run(["--gpus", "4", "--tp", "2", *TINY], env_extra={"BENCH_FAIL_RANK": "1"}, timeout=300)
    assert r.returncode != 0
    assert "rank 1 exited with 3" in r.stderr
    assert _json_lines(r.stdout) == []
    assert time.time() - t0 < 120


@pytest.mark.parametrize("sp", [False, True])
def test_bench_tp_comm_chunks_gloo(sp):
    """TP2 (optionally + sequence parallel) with the row-parallel output collectives in 2 overlapped pieces gives the
    loss of the one-piece run; the JSON carries the layout's communication estimate."""
    extra = ["--sequence-parallel"] if sp else []
    losses = {}
    for c in ("1", "2"):
        r = _run(["--gpus", "2", "--tp", "2", "--tp-comm-chunks", c, *extra, *TINY])
        assert r.returncode == 0, r.stderr[-4000:]
        res = _json_lines(r.stdout)[0]
        losses[c] = res["config"]["loss"]
        est = res["config"]["comm_estimate"]
        assert est["tp_bytes"] > 0 and est["dp_bytes"] == 0 and est["pp_bytes"] == 0
    assert losses["2"] == pytest.approx(losses["1"], rel=1e-5)


@pytest.mark.parametrize("extra", [[], ["--tp-comm-chunks", "2"], ["--grad-acc", "2", "--gpus", "4", "--pp", "2"]])
def test_bench_sp_gather_overlap_gloo(extra):
    """Sequence parallelism with the norm's all-gather folded into (and overlapped with) the q/k/v and gate/up GEMMs
    (SCALING_AMD_SP_OVERLAP=1, default) trains to the losses and parameters of the gather-in-the-norm path."""
    losses = {}
    for mode in ("0", "1"):
        args = ["--tp", "2", "--sequence-parallel", *TINY, *extra]
        if "--gpus" not in extra:
            args = ["--gpus", "2", *args]
        r = _run(args, env_extra={"SCALING_AMD_SP_OVERLAP": mode})
        assert r.returncode == 0, r.stderr[-4000:]
        res = _json_lines(r.stdout)[0]
        losses[mode] = (res["config"]["loss"], res["config"].get("param_checksum"))
    assert losses["1"][0] == pytest.approx(losses["0"][0], rel=1e-5)
    if losses["0"][1] is not None:
        assert losses["1"][1] == pytest.approx(losses["0"][1], rel=1e-4)


@pytest.mark.parametrize("preset,gpus,tp,pp,dp,acc,ac,sp,lora", [
    ("baseline3", 8, 2, 1, 4, 1, "disabled", True, False),
    ("baseline4", 8, 2, 2, 2, 4, "every_layer", True, False),
    ("baseline4_save_matmuls", 8, 2, 2, 2, 4, "every_layer_save_matmuls", True, False),
    ("baseline5", 8, 1, 1, 8, 1, "disabled", False, True),
    ("baseline3", 4, 2, 1, 2, 1, "disabled", True, False),
])
def test_bench_preset_layouts(preset, gpus, tp, pp, dp, acc, ac, sp, lora):
    """``--preset`` pins BASELINE.json configs 3-5 to their topology (TP x PP x DP, ZeRO-1, activation
    checkpointing, sequence parallelism, LoRA) for any GPU count the layout divides."""
    sys.path.insert(0, ROOT)
    import bench

    a = bench._args(["--gpus", str(gpus), "--preset", preset])
    t = bench._config_dict(a, gpus, 0, 0)["topology"]
    assert (t["model_parallel_size"], t["pipe_parallel_size"], t["data_parallel_size"]) == (tp, pp, dp)
    assert t["gradient_accumulation_steps"] == acc and t["activation_checkpointing_type"] == ac
    assert t["sequence_parallel"] is sp and bool(a.lora) is lora and a.zero == 1
    cfg = bench._config_dict(a, gpus, 0, 0)
    assert ("lora_config" in cfg["transformer_architecture"]) is lora
    with pytest.raises(SystemExit):
        bench._args(["--gpus", "1", "--preset", "baseline4"])


def test_bench_preset_rejects_conflicting_flags():
    """An explicit layout flag that the preset would silently overwrite is an error; one that agrees is fine."""
    sys.path.insert(0, ROOT)
    import bench

    with pytest.raises(SystemExit, match="micro-batch"):
        bench._args(["--gpus", "8", "--preset", "baseline4", "--micro-batch", "2"])
    with pytest.raises(SystemExit, match="tp"):
        bench._args(["--gpus", "8", "--preset", "baseline3", "--tp=4"])
    a = bench._args(["--gpus", "8", "--preset", "baseline4", "--micro-batch", "4", "--steps", "3"])
    assert a.micro_batch == 4 and a.steps == 3


def test_bench_preset_runs_gloo():
    """The TP2 x PP2 preset (BASELINE #4) end to end on 4 CPU ranks; the JSON names the preset."""
    r = _run(["--gpus", "4", "--preset", "baseline4", "--model", "llama_tiny", "--backend", "gloo", "--seq-len", "64",
              "--steps", "1", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-4000:]
    res = _json_lines(r.stdout)[0]
    assert res["config"]["preset"] == "baseline4"
    assert res["config"]["parallelism"].startswith("tp2_pp2_dp1_zero1_ac-every_layer_sp")


def test_default_tp_comm_chunks():
    """Auto ``--tp-comm-chunks``: 1 without TP or for short micro-batches (pieces would fall under 2048 tokens),
    more pieces when the TP collective is long enough to hide behind the GEMM."""
    from scaling_amd.transformer.utils.comm_estimate import default_tp_comm_chunks as f

    assert f(hidden_size=4096, tokens=8 * 4096, tp=1) == 1
    assert f(hidden_size=4096, tokens=2048, tp=2) == 1
    assert f(hidden_size=4096, tokens=8 * 2048, tp=2) == 4
    assert f(hidden_size=4096, tokens=4 * 2048, tp=2) == 2
    sys.path.insert(0, ROOT)
    import bench

    a = bench._args(["--gpus", "2", "--preset", "baseline3"])
    assert a.tp_comm_chunks == 0  # resolved when the config is built
    cfg = bench._config_dict(a, 2, 0, 0)
    assert cfg["topology"]["tensor_parallel_comm_chunks"] == a.tp_comm_chunks >= 2


@pytest.mark.parametrize("preset,ac", [("baseline3", None), ("baseline4", None),
                                       ("baseline4", "every_layer_save_matmuls")])
def test_bench_shard_proxy_gloo(preset, ac):
    """``--shard-proxy``: one process runs rank 0's TP2 shard of the preset (one pipeline stage's layers) with stubbed
    collectives; the JSON says it is a per-rank proxy (not the headline), on one device, with the preset's layout
    (an explicit --activation-checkpointing wins for the checkpointing A/B)."""
    args = ["--shard-proxy", preset, "--model", "llama_tiny", "--backend", "gloo", "--seq-len", "64", "--steps", "1",
            "--warmup", "1"] + (["--activation-checkpointing", ac] if ac else [])
    r = _run(args, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    res = _json_lines(r.stdout)[0]
    assert res["metric"].startswith("per-rank proxy") and res["n_gpus"] == 1 and res["vs_baseline"] is None
    c = res["config"]
    assert c["shard_proxy"] == preset and c["tp"] == 2 and c["pp"] == 1 and c["dp"] == 1 and c["sequence_parallel"]
    assert c["activation_checkpointing"] == (ac or ("every_layer" if preset == "baseline4" else "disabled"))
    assert c["micro_batch"] == (4 if preset == "baseline4" else 8) and math.isfinite(c["loss"])
    assert c["proxy_8gpu_tokens_s_without_comm"] > 0


def test_bench_shard_proxy_emulated_comm_flag_gloo():
    """``--proxy-comm emulate`` is accepted and reported (on CPU ranks the emulation is a no-op: it costs GPU time only)."""
    r = _run(["--shard-proxy", "baseline3", "--proxy-comm", "emulate", "--model", "llama_tiny", "--backend", "gloo",
              "--seq-len", "64", "--steps", "1", "--warmup", "1"], timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    res = _json_lines(r.stdout)[0]
    assert res["config"]["proxy_comm"] == "emulate" and "emulated" in res["metric"]


def test_collective_time_model():
    """The xGMI model: one direction of one link is 76.8 GB/s (153.6 GB/s bidirectional); a TP2 all-reduce of the 7B
    [32768, 4096] bf16 activations sends its size once over the pair's one link, a DP8 ring spreads over 7 links."""
    from scaling_amd.transformer.utils import comm_estimate as ce

    assert ce.XGMI_LINK_BYTES_PER_S == 76.8e9
    nb = 32768 * 4096 * 2
    assert ce.ring_send_bytes("all_reduce", nb, 2) == nb
    assert ce.ring_send_bytes("reduce_scatter", nb, 8) == pytest.approx(nb * 7 / 8)
    t2 = ce.collective_time_s("all_reduce", nb, 2, link_efficiency=1.0)
    assert t2 == pytest.approx(ce.COLLECTIVE_LATENCY_S + nb / 76.8e9)
    t8 = ce.collective_time_s("all_reduce", nb, 8, link_efficiency=1.0)
    assert t8 == pytest.approx(ce.COLLECTIVE_LATENCY_S + 2 * nb * 7 / 8 / (7 * 76.8e9))
    assert ce.collective_time_s("all_reduce", nb, 1) == 0.0


@pytest.mark.parametrize("split,gpus,backend,ndev,want", [
    ("1", 2, "gloo-gpu", 1, ["0:0-127", "0:128-255"]),
    ("256", 4, "gloo-gpu", 1, ["0:0-63", "0:64-127", "0:128-191", "0:192-255"]),
    ("1", 4, "gloo-gpu", 2, ["0:0-127", "1:0-127", "0:128-255", "1:128-255"]),  # ranks dealt over 2 visible devices
    ("1", 2, "gloo", 1, [None, None]), ("0", 2, "gloo-gpu", 1, [None, None])])
def test_bench_launcher_cu_split(monkeypatch, split, gpus, backend, ndev, want):
    """SCALING_AMD_REHEARSAL_CU_SPLIT gives each rehearsal rank a disjoint CU range (HSA_CU_MASK) of the device it runs
    on (rank % visible devices), only for the GPU-sharing gloo-gpu backend."""
    import argparse

    import bench

    envs = []

    class _Proc:
        def __init__(self, argv, env):
            envs.append(env)

        def poll(self):
            return 0

    monkeypatch.setenv("SCALING_AMD_REHEARSAL_CU_SPLIT", split)
    monkeypatch.delenv("HSA_CU_MASK", raising=False)
    monkeypatch.setattr(bench.subprocess, "Popen", _Proc)
    monkeypatch.setattr(bench.signal, "signal", lambda *a: None)
    monkeypatch.setattr(bench, "_visible_devices", lambda: ndev)
    a = argparse.Namespace(gpus=gpus, backend=backend, launch_timeout=10)
    assert bench._launch(a) == 0
    assert [e.get("HSA_CU_MASK") for e in envs] == want


def test_bench_transformer_example_args():
    """``--model transformer_example`` (BASELINE #2) takes the example config's micro-batching and sequence length and
    turns the 7B TunableOp table off; explicit flags win."""
    sys.path.insert(0, ROOT)
    import bench

    cfg = bench.example_config()
    a = bench._args(["--model", "transformer_example"])
    assert a.micro_batch == cfg["topology"]["micro_batch_size"]
    assert a.grad_acc == cfg["topology"]["gradient_accumulation_steps"]
    assert a.seq_len == cfg["transformer_architecture"]["sequence_length"] and a.gemm_tuning == "off"
    b = bench._args(["--model", "transformer_example", "--seq-len", "32", "--gemm-tuning", "use"])
    assert b.seq_len == 32 and b.gemm_tuning == "use"
