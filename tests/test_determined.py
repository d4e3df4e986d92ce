"""Determined-cluster trainer paths against a duck-typed cluster (reference trainer.py:317-558;
``determined`` itself is not installed, so parity with the real client is unpinned): checkpoint storage
through ``store_path``, metric reporting, preemption save + exit, resume from the trial's
``latest_checkpoint``, deletion of preemption checkpoints off the save grid and of older optimizer states."""
from __future__ import annotations

import contextlib
import os
import uuid
from pathlib import Path
from types import SimpleNamespace

import pytest

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.cpu


class FakeCheckpoint:
    def __init__(self, root: Path, uid: str, steps: int):
        self.uuid, self.metadata, self.state = uid, {"steps_completed": steps}, "CheckpointState.COMPLETED"
        self.root = root
        self.deleted = False
        self.removed: list = []

    def delete(self):
        self.deleted = True

    def remove_files(self, globs):
        self.removed.extend(globs)
        for g in globs:
            for f in (self.root / self.uuid).glob(g):
                f.unlink()


class FakeCluster:
    """checkpoint.store_path / restore_path, distributed.broadcast, preempt, train.report_*."""

    def __init__(self, root: Path, preempt_at: int | None = None):
        self.root, self.preempt_at = root, preempt_at
        self.ckpts: list[FakeCheckpoint] = []
        self.reported: list = []
        self.iter_fn = lambda: 0
        cluster = self

        class _Ckpt:
            @contextlib.contextmanager
            def store_path(self, metadata):
                uid = str(uuid.uuid4())
                p = cluster.root / uid
                p.mkdir(parents=True)
                yield p, uid
                cluster.ckpts.append(FakeCheckpoint(cluster.root, uid, metadata["steps_completed"]))

            @contextlib.contextmanager
            def restore_path(self, uid):
                yield cluster.root / uid

        self.checkpoint = _Ckpt()
        self.distributed = SimpleNamespace(broadcast=lambda x: x, get_rank=lambda: 0, get_local_rank=lambda: 0)
        self.preempt = SimpleNamespace(should_preempt=lambda: preempt_at is not None and self.iter_fn() >= preempt_at)
        self.train = SimpleNamespace(
            report_training_metrics=lambda steps_completed, metrics: self.reported.append(("train", steps_completed)),
            report_validation_metrics=lambda steps_completed, metrics: self.reported.append(("val", steps_completed)))


def _scenario(tmp: str, preempt_at, latest, save_interval: int, iters: int, delete_opt: bool, existing: list):
    import scaling_amd.transformer.train as T
    from scaling_amd.core.runner.launch_config import LaunchConfig
    from tests.test_training import _config, _make_data

    os.environ["DETERMINED_TEST"] = "True" if preempt_at is not None else "False"
    tmp_p = Path(tmp)
    if not (tmp_p / "data.bin").exists():
        _make_data(tmp_p / "data")
    cluster = FakeCluster(tmp_p / "det", preempt_at)
    cluster.ckpts = [FakeCheckpoint(tmp_p / "det", u, s) for u, s in existing]
    info = SimpleNamespace(latest_checkpoint=latest, trial=SimpleNamespace(trial_id=1))
    T.TransformerTrainer._cluster_info = lambda self: info
    T.TransformerTrainer._trial_checkpoints = lambda self: list(cluster.ckpts)
    profiler = SimpleNamespace(batches=[], update_batch_idx=lambda i: profiler.batches.append(i))
    cfg = _config(tmp_p, 1, 1, 1)
    cfg["runner"] = {"use_determined": True}
    cfg["trainer"].update(save_dir=None, load_dir=None, save_interval=save_interval, train_iterations=iters,
                          delete_past_optimizer_states=delete_opt, assert_checkpoint_loaded=latest is not None)
    orig = T.TransformerTrainer.train_step

    def step(self):
        out = orig(self)
        cluster.iter_fn = lambda: self.context.iterations
        return out

    T.TransformerTrainer.train_step = step
    metrics = T.main(LaunchConfig.from_launcher_args([]), overwrite_config=cfg, return_metrics=True,
                     determined_context=cluster, determined_profiler=profiler)
    return {
        "losses": [m["training/loss"] for m in metrics],
        "ckpts": [(c.uuid, c.metadata["steps_completed"], c.deleted, list(c.removed)) for c in cluster.ckpts],
        "reported": cluster.reported, "profiled": profiler.batches,
        "files": {c.uuid: sorted(p.name for p in (tmp_p / "det" / c.uuid).rglob("*.pt")) for c in cluster.ckpts
                  if (tmp_p / "det" / c.uuid).exists()},
    }


def _run(tmp_path, **kw):
    return run_distributed(_scenario, 1, tmp=str(tmp_path), **kw)[0]


def test_determined_store_report_and_delete_old_optimizer_states(tmp_path):
    r = _run(tmp_path, preempt_at=None, latest=None, save_interval=2, iters=6, delete_opt=True, existing=[])
    assert len(r["losses"]) == 6
    assert [c[1] for c in r["ckpts"]] == [2, 4, 6]
    assert r["reported"] == [("train", i) for i in range(1, 7)]
    assert r["profiled"] == list(range(6))
    # every checkpoint but the newest lost its optimizer states, the newest keeps them
    uids = [c[0] for c in r["ckpts"]]
    for u in uids[:-1]:
        assert not any("optimizer_state" in f for f in r["files"][u]) and any("model_state" in f for f in r["files"][u])
    assert any("optimizer_state" in f for f in r["files"][uids[-1]])


def test_determined_preemption_then_resume_from_latest(tmp_path):
    full = _run(tmp_path, preempt_at=None, latest=None, save_interval=100, iters=6, delete_opt=False, existing=[])
    pre = _run(tmp_path, preempt_at=3, latest=None, save_interval=100, iters=6, delete_opt=False, existing=[])
    assert len(pre["losses"]) == 2 and [c[1] for c in pre["ckpts"]] == [3]  # saved at preemption, loop left
    uid = pre["ckpts"][0][0]
    res = _run(tmp_path, preempt_at=None, latest=uid, save_interval=100, iters=6, delete_opt=False,
               existing=[(uid, 3)])
    # the resumed trial continues at step 4 with the restored optimizer + data position: same losses
    assert res["losses"] == full["losses"][3:]
    assert res["profiled"] == [3, 4, 5]


def test_determined_deletes_preemption_checkpoints_off_grid(tmp_path):
    existing = [("a", 2), ("b", 3), ("c", 4), ("d", 5)]
    r = _run(tmp_path, preempt_at=None, latest=None, save_interval=2, iters=0, delete_opt=False, existing=existing)
    deleted = {u for u, _, d, _ in r["ckpts"] if d}
    assert deleted == {"b"}  # 5 is off-grid too but is the newest: kept for resuming
