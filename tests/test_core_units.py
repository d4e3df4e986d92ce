"""CPU unit tests of core algorithms (reference: tests/core/test_data/test_file_handles.py,
test_blended_dataset_weights.py, test_broadcast_data.py, test_optimizer/test_learning_rate_scheduler.py,
test_nn/test_pipeline_partitioning.py, test_logging/test_logger_config.py, test_nn/test_attention_helpers.py,
tests/transformer/test_data_utils.py, test_training/test_parameters_count.py, test_topology/test_topology.py)."""
from errno import ESTALE
from unittest import mock

import numpy as np
import pytest
import torch

from tests.dist_utils import make_topology, run_distributed

pytestmark = pytest.mark.cpu


# ---------------------------------------------------------------- file handles (fault injection)
class _FlakyFile:
    def __init__(self, fail_times: int, exc_factory) -> None:
        self.attempt = 0
        self.fail_times = fail_times
        self.exc_factory = exc_factory

    def open(self, *args, **kwargs):
        self.attempt += 1
        return self

    def close(self):
        pass

    def read(self, *args, **kwargs):
        if self.attempt > self.fail_times:
            return b"ok"
        raise self.exc_factory()


def _stale():
    e = OSError()
    e.errno = ESTALE
    e.strerror = "Stale file handle"
    return e


@pytest.mark.parametrize("factory", ["stale", "retryable"])
def test_file_handle_retries_then_succeeds(factory):
    from scaling_amd.core.data.file_handles import FileHandle, RetryableException

    f = _FlakyFile(4, _stale if factory == "stale" else (lambda: RetryableException("flaky")))
    fh = FileHandle("any/path")
    with mock.patch("builtins.open", f.open), mock.patch("time.sleep"):
        assert fh.retry_operation(lambda h: h.read(), max_delay=0) == b"ok"
    assert f.attempt == 5


def test_file_handle_gives_up_and_does_not_retry_other_errors():
    from scaling_amd.core.data.file_handles import FileHandle

    f = _FlakyFile(100, _stale)
    with mock.patch("builtins.open", f.open), mock.patch("time.sleep"):
        with pytest.raises(Exception, match="Stale file handle even after 5 retries"):
            FileHandle("p").retry_operation(lambda h: h.read(), max_delay=0)
    g = _FlakyFile(100, lambda: ValueError("boom"))
    with mock.patch("builtins.open", g.open):
        with pytest.raises(ValueError):
            FileHandle("p").retry_operation(lambda h: h.read())
    assert g.attempt == 1


# ---------------------------------------------------------------- blended dataset weights
NUM_DOCS = [[900, 1], [900, 900], [900, 50, 40, 100], [900, 50, 40, 100, 1], [25000, 200, 200]]


@pytest.mark.parametrize("num_docs", NUM_DOCS)
def test_weights_alpha0_equalises_and_alpha1_is_identity(num_docs):
    from scaling_amd.core.data.blended_dataset import weights_by_num_docs

    w0 = weights_by_num_docs(num_docs, alpha=0.0)
    weighted = [n * w for n, w in zip(num_docs, w0)]
    assert all(round(x, 4) == round(weighted[0], 4) for x in weighted)
    w1 = weights_by_num_docs(num_docs, alpha=1.0)
    wn = [n * w for n, w in zip(num_docs, w1)]
    assert np.allclose(np.array(wn) / sum(wn), np.array(num_docs) / sum(num_docs), atol=1e-4)


@pytest.mark.parametrize("num_docs", NUM_DOCS[2:4])
@pytest.mark.parametrize("alpha", [0.2, 0.5, 0.8])
def test_weights_move_towards_identity_with_alpha(num_docs, alpha):
    from scaling_amd.core.data.blended_dataset import weights_by_num_docs

    w1 = weights_by_num_docs(num_docs, alpha=1.0)
    wa = weights_by_num_docs(num_docs, alpha=alpha)
    wb = weights_by_num_docs(num_docs, alpha=alpha - 0.1)
    assert all(abs(a - c) < abs(b - c) for a, b, c in zip(wa, wb, w1))


def test_weights_examples_proportional():
    from scaling_amd.core.data.blended_dataset import weights_examples_proportional

    def probs(w, e):  # per-sample weights -> dataset sampling probabilities
        x = np.array(w) * np.array(e)
        return x / x.sum()

    e = [100, 300]
    assert np.allclose(probs(weights_examples_proportional(e, temperature=1.0), e), [0.25, 0.75])
    assert np.allclose(probs(weights_examples_proportional(e, temperature=1.0, maximum=100), e), [0.5, 0.5])
    hot = probs(weights_examples_proportional(e, temperature=2.0), e)
    assert 0.25 < hot[0] < 0.5  # temperature flattens towards uniform


# ---------------------------------------------------------------- learning-rate schedule
@pytest.mark.parametrize("style", ["linear", "constant", "cosine"])
@pytest.mark.parametrize("warmup", [0, 5])
@pytest.mark.parametrize("train_iters", [4, 10, 20])
def test_learning_rate_schedule_shape(style, warmup, train_iters):
    from scaling_amd.core import LearningRateScheduler, LearningRateSchedulerConfig

    cfg = LearningRateSchedulerConfig(learning_rate=0.01, learning_rate_minimum=0.001, learning_rate_decay_style=style,
                                      learning_rate_decay_iters=10, learning_rate_warmup_steps=warmup)
    sched = LearningRateScheduler(config=cfg)
    prev = cfg.learning_rate if warmup == 0 else 0.0
    for step in range(1, train_iters + 1):
        lr = sched.get_lr(step_index=step)
        if step < warmup:
            assert lr > prev
        elif style == "constant" and step > warmup:
            assert lr == cfg.learning_rate
        elif warmup < step < cfg.learning_rate_decay_iters and style != "constant":
            assert lr < prev
        elif step > cfg.learning_rate_decay_iters and style != "constant":
            assert lr == cfg.learning_rate_minimum
        prev = lr


# ---------------------------------------------------------------- pipeline partitioning
@pytest.mark.parametrize("pp", [1, 2, 3, 5, 17, 32])
@pytest.mark.parametrize("layers", [1, 2, 5, 17, 32, 73, 128])
def test_pipe_partition_uniform(pp, layers):
    from scaling_amd.core import pipe_partition_uniform

    if layers < pp:
        with pytest.raises(AssertionError):
            pipe_partition_uniform(item_count=layers, partition_count=pp)
        return
    parts = pipe_partition_uniform(item_count=layers, partition_count=pp)
    lengths = [p.length for p in parts]
    assert len(parts) == pp and min(lengths) > 0 and max(lengths) - min(lengths) <= 1 and sum(lengths) == layers
    assert all(parts[i].end == parts[i + 1].start for i in range(pp - 1))


@pytest.mark.parametrize("weights,pp", [([5, 1, 1, 1, 1, 5], 2), ([1] * 10, 3), ([10, 1, 1, 1, 10, 1, 1, 1], 4)])
def test_pipe_partition_balanced_minimises_bottleneck(weights, pp):
    import itertools

    from scaling_amd.core.nn.parallel_module.pipeline_partitioning import partition_balanced_weights

    parts = partition_balanced_weights(weights, pp)
    assert len(parts) == pp and parts[0].start == 0 and parts[-1].end == len(weights)
    got = max(sum(weights[p.start : p.end]) for p in parts)
    best = min(
        max(sum(weights[a:b]) for a, b in zip((0,) + cuts, cuts + (len(weights),)))
        for cuts in itertools.combinations(range(1, len(weights)), pp - 1)
    )
    assert got == best


def test_pipe_partition_from_indices():
    from scaling_amd.core.nn.parallel_module.pipeline_partitioning import pipe_partition_from_indices

    parts = pipe_partition_from_indices([0, 3, 7, 10], num_layers=10)
    assert [(p.start, p.end) for p in parts] == [(0, 3), (3, 7), (7, 10)]


# ---------------------------------------------------------------- logger config
def test_logger_config_adds_date_and_checks_wandb(tmp_path, monkeypatch):
    from scaling_amd.core.logging import LoggerConfig

    c = LoggerConfig(log_dir=str(tmp_path / "logs"))
    assert c.log_dir is not None and c.log_dir.parent == tmp_path / "logs"
    again = LoggerConfig(**{**c.model_dump(), "log_dir": str(c.log_dir)})
    assert again.log_dir == c.log_dir  # a dated directory is not re-dated
    monkeypatch.delenv("WANDB_API_KEY", raising=False)
    with pytest.raises(Exception):
        LoggerConfig(use_wandb=True, wandb_ranks=[0])
    assert LoggerConfig(metrics_ranks=[0, 3]).is_rank_in_metrics_ranks(3)
    assert not LoggerConfig(metrics_ranks=[0]).is_rank_in_metrics_ranks(1)


# ---------------------------------------------------------------- attention helpers / data utils
def test_dense_mask_from_cumulative_seq_lengths():
    from scaling_amd.core.nn.attention import cumulative_seq_lengths_to_dense_attention_mask

    cu = torch.tensor([0, 2, 4, 7, 8])
    m = cumulative_seq_lengths_to_dense_attention_mask(cu, 4, causal=True)
    assert m.shape == (2, 1, 4, 4)
    allowed = ~m[:, 0]
    exp0 = torch.tensor([[1, 0, 0, 0], [1, 1, 0, 0], [0, 0, 1, 0], [0, 0, 1, 1]], dtype=torch.bool)
    exp1 = torch.tensor([[1, 0, 0, 0], [1, 1, 0, 0], [1, 1, 1, 0], [0, 0, 0, 1]], dtype=torch.bool)
    assert torch.equal(allowed[0], exp0) and torch.equal(allowed[1], exp1)
    nc = ~cumulative_seq_lengths_to_dense_attention_mask(cu, 4, causal=False)[:, 0]
    assert torch.equal(nc[0], torch.tensor([[1, 1, 0, 0], [1, 1, 0, 0], [0, 0, 1, 1], [0, 0, 1, 1]], dtype=torch.bool))


def test_repeat_kv_and_max_seq_length():
    from scaling_amd.core.nn.attention import get_max_seq_length, repeat_kv

    x = torch.arange(2 * 3 * 4).view(2, 3, 4).float()
    r = repeat_kv(x, 2)
    assert r.shape == (2, 6, 4) and torch.equal(r[:, 0], r[:, 1]) and torch.equal(r[:, 2], x[:, 1])
    assert get_max_seq_length(torch.tensor([0, 3, 10, 12])) == 7


def test_cu_seqlens_and_position_ids_reset_at_eod():
    from scaling_amd.transformer.data.utils import get_cumulative_seq_lengths, get_position_ids

    ids = torch.tensor([[5, 0, 7, 8, 0, 9], [1, 2, 3, 4, 5, 6]])
    cu = get_cumulative_seq_lengths(ids, reset_attention_mask=True)
    assert cu.tolist() == [0, 2, 5, 6, 12]
    assert get_cumulative_seq_lengths(ids, reset_attention_mask=False).tolist() == [0, 6, 12]
    pos = get_position_ids(ids, reset_position_ids=True)
    assert pos.tolist() == [[0, 1, 0, 1, 2, 0], [0, 1, 2, 3, 4, 5]]
    assert get_position_ids(ids, reset_position_ids=False).tolist() == [list(range(6))] * 2


# ---------------------------------------------------------------- broadcast_data / topology (gloo, 2 ranks)
def _broadcast_body():
    from scaling_amd.core.data.broadcast_data import broadcast_data

    topo = make_topology(model_parallel_size=2)
    if topo.model_parallel_rank == 0:
        ts = [torch.arange(12).view(3, 4), torch.arange(5), torch.ones(2, 2, 2, dtype=torch.long)]
    else:
        ts = [None, None, None]
    out = broadcast_data(ts, torch.long, topo)
    return [t.tolist() for t in out]


def test_broadcast_data_over_model_parallel_group():
    res = run_distributed(_broadcast_body, world_size=2)
    assert res[0] == res[1]
    assert res[1][0] == torch.arange(12).view(3, 4).tolist() and res[1][1] == list(range(5))


def _topology_body():
    topo = make_topology(model_parallel_size=2, pipe_parallel_size=2)
    return dict(rank=topo.config.global_rank, mp=topo.model_parallel_rank, pp=topo.pipe_parallel_rank,
                dp=topo.data_parallel_rank, io=topo.is_io_rank,
                peer=topo.get_global_rank(pipe_parallel_rank=1 - topo.pipe_parallel_rank))


def test_topology_rank_layout_world4():
    """mp fastest, then dp, then pp (reference topology.py:45-55); IO ranks = first/last stage, mp 0."""
    res = run_distributed(_topology_body, world_size=4)
    for r, d in res.items():
        assert (d["mp"], d["dp"], d["pp"]) == (r % 2, 0, r // 2)
        assert d["io"] == (d["mp"] == 0)
        assert d["peer"] == (r + 2) % 4


def _param_count_body(mp, pp):
    from scaling_amd.transformer.context import TransformerConfig, TransformerContext
    from scaling_amd.transformer.model import init_model

    import os

    world = int(os.environ["WORLD_SIZE"])
    cfg = TransformerConfig.from_dict({
        "topology": {"world_size": world, "global_rank": int(os.environ["RANK"]), "local_slot": int(os.environ["RANK"]),
                     "model_parallel_size": mp, "pipe_parallel_size": pp, "micro_batch_size": 1,
                     "gradient_accumulation_steps": 2},
        "transformer_architecture": {"vocab_size": 256, "hidden_size": 32, "num_layers": 4, "num_attention_heads": 4,
                                     "sequence_length": 16, "precision": "float32", "weight_tying": True},
    })
    from scaling_amd.core import Topology

    topo = Topology(config=cfg.topology)
    ctx = TransformerContext(config=cfg, topology=topo)
    ctx.initialize(master_addr="127.0.0.1", master_port=os.environ["MASTER_PORT"], seed=42)
    model = init_model(context=ctx)
    return model.get_params_count()


@pytest.mark.parametrize("mp,pp", [(2, 1), (1, 2)])
def test_parameter_count_independent_of_layout(mp, pp):
    """Reference test_parameters_count.py: total / unique parameter counts do not depend on TP/PP."""
    base = run_distributed(_param_count_body, world_size=1, mp=1, pp=1)[0]
    other = run_distributed(_param_count_body, world_size=2, mp=mp, pp=pp)
    for r in other.values():
        assert r[1] == base[1]


# ---------------------------------------------------------------- hang watchdog
def test_hang_watchdog_dumps_stacks_on_stall(tmp_path):
    import time

    from scaling_amd.core.utils.watchdog import HangWatchdog

    seen = []
    wd = HangWatchdog(0.3, rank=3, log_dir=tmp_path, on_hang=seen.append, poll_s=0.05)
    for _ in range(5):  # steady heartbeats: no report
        time.sleep(0.05)
        wd.heartbeat()
    assert wd.fired == 0
    time.sleep(0.6)  # stall
    wd.stop()
    assert wd.fired >= 1 and seen and seen[0] >= 0.3
    dump = (tmp_path / "hang_rank3.txt").read_text()
    assert "no progress" in dump and "test_hang_watchdog_dumps_stacks_on_stall" in dump
