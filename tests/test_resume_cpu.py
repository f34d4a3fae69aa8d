"""Resume continues the run.

The reference loop being resumed is ``mnist_sync/worker.py:58-72``: ``for batch_cnt in
range(500)`` with the batch slice, the dropout draw and the every-10-steps eval all keyed by
the position in the epoch.  A job stopped after k steps (``max_steps``), checkpointed, and
resumed must be the uninterrupted job: same parameters and optimizer state bit for bit (sync,
CPU), the same PS step counters (async), and the same cadence of reference print lines.
"""
import os

import pytest
import torch

from conftest import free_port
from dist_helpers import spawn, train_rank

STEPS = 6
CUT = 3


def _cfg(tmp, **kw):
    base = dict(mode="sync", shard="contiguous", num_ps=3, steps=STEPS, batch_size=20,
                eval_every=2, engine="torch", quiet=False, checkpoint_dir=str(tmp))
    base.update(kw)
    return base


def _train(cfg_kw):
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import synthetic_mnist
    tr = Trainer(TrainConfig(**cfg_kw), DistEnv(), dataset=synthetic_mnist(400, 100, seed=11))
    tr.train()
    return tr


def _progress(out):
    return [ln.rsplit(" accuracy:", 1)[0] for ln in out.splitlines() if "batch:" in ln]


def test_sync_resume_is_bit_identical_to_the_uninterrupted_run(tmp_path, capsys):
    full = _train(_cfg(tmp_path / "full"))
    out_full = capsys.readouterr().out
    part = _train(_cfg(tmp_path / "cut", max_steps=CUT))
    out_a = capsys.readouterr().out
    assert part.global_step == CUT
    res = _train(_cfg(tmp_path / "cut", resume=True))
    out_b = capsys.readouterr().out
    assert res.global_step == STEPS
    assert torch.equal(res.params, full.params)
    for p, ps in full.servers.items():
        q = res.servers[p]
        assert q.t == ps.t == STEPS
        assert torch.equal(q.m, ps.m) and torch.equal(q.v, ps.v)
    # the reference lines: evals at batch 0, 2, 4 exactly once across the two runs
    assert _progress(out_a) + _progress(out_b) == _progress(out_full)
    assert _progress(out_full) == [f"epoch: 0 batch: {c}" for c in (0, 2, 4)] or \
        _progress(out_full) == [f"Worker0 epoch: 0 batch: {c}" for c in (0, 2, 4)]
    # the resumed run's eval history continues at the right global steps with equal accuracy
    assert [h["step"] for h in res.history] == [5]
    assert [h["acc"] for h in res.history] == [h["acc"] for h in full.history if h["step"] == 5]


def test_resume_across_epochs_skips_finished_epochs(tmp_path):
    full = _train(_cfg(tmp_path / "full", epochs=2, steps=3, eval_every=0, quiet=True))
    _train(_cfg(tmp_path / "cut", epochs=2, steps=3, eval_every=0, quiet=True, max_steps=4))
    res = _train(_cfg(tmp_path / "cut", epochs=2, steps=3, eval_every=0, quiet=True, resume=True))
    assert res.global_step == 6
    assert torch.equal(res.params, full.params)


def _dist_run(tmp, world, **kw):
    os.makedirs(tmp, exist_ok=True)
    spawn(train_rank, world, free_port(), kw, str(tmp))
    return [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=False)
            for r in range(world)]


@pytest.mark.slow
def test_sync_w2_resume_matches_uninterrupted(tmp_path):
    base = dict(mode="sync", shard="flat", steps=STEPS, batch_size=20, eval_every=0,
                quiet=True, engine="torch", watchdog_s=120.0, data_sharding="stride")
    full = _dist_run(tmp_path / "full", 2, **base, checkpoint_dir=str(tmp_path / "ckf"))
    _dist_run(tmp_path / "a", 2, **base, checkpoint_dir=str(tmp_path / "ck"), max_steps=CUT)
    res = _dist_run(tmp_path / "b", 2, **base, checkpoint_dir=str(tmp_path / "ck"), resume=True)
    for r in range(2):
        assert torch.equal(res[r]["params"], full[r]["params"])
        assert res[r]["ps_t"] == full[r]["ps_t"]
        assert res[r]["summary"]["steps"] == STEPS


@pytest.mark.slow
def test_async_w2_resume_continues_ps_step_counters(tmp_path):
    """Async: arrival order makes the parameters run-dependent, but every PS must end with
    one Adam step per push of the whole job (W x steps), the resumed run serving exactly the
    pushes after the cut, each worker's in order (provenance check on)."""
    base = dict(mode="async", shard="contiguous", steps=STEPS, batch_size=20, eval_every=0,
                quiet=True, engine="torch", watchdog_s=120.0, check_provenance=True)
    _dist_run(tmp_path / "a", 2, **base, checkpoint_dir=str(tmp_path / "ck"), max_steps=CUT)
    res = _dist_run(tmp_path / "b", 2, **base, checkpoint_dir=str(tmp_path / "ck"), resume=True)
    ps_t = {}
    for r, rec in enumerate(res):
        ps_t.update(rec["ps_t"])
        assert len(rec["provenance"]) == (STEPS - CUT)  # one hosted PS, one remote worker
        assert rec["summary"]["steps"] == STEPS and rec["summary"]["images"] == (STEPS - CUT) * 20
        assert torch.isfinite(rec["params"]).all()
    assert ps_t == {0: 2 * STEPS, 1: 2 * STEPS}


def test_resume_from_manifest_without_ps_segments_keeps_ps_counters(tmp_path, capsys):
    """A manifest written before round 5 has no ``ps_segments``: resuming it with the same
    policy and PS count restores every PS's own step counter (Adam's bias correction) instead of
    resetting them all to the global step, and says so."""
    import glob
    import json
    full = _train(_cfg(tmp_path / "full"))
    _train(_cfg(tmp_path / "cut", max_steps=CUT))
    mans = glob.glob(os.path.join(str(tmp_path / "cut"), "**", "manifest.json"), recursive=True)
    assert mans
    for mp in mans:
        man = json.load(open(mp))
        man.pop("ps_segments", None)
        json.dump(man, open(mp, "w"))
    capsys.readouterr()
    res = _train(_cfg(tmp_path / "cut", resume=True))
    err = capsys.readouterr().err
    assert "no ps_segments" in err
    assert torch.equal(res.params, full.params)
    for p, ps in full.servers.items():
        assert res.servers[p].t == ps.t == STEPS
