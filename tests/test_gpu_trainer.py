"""End-to-end Trainer paths on one MI355X with the HIP engine (native extension loaded).

* sync training through the native SyncRunner: checkpoint -> resume reproduces the exact
  continuation (params, Adam state, PS step counters) of an uninterrupted run;
* async mode (W = 1: local whole-shard updates) and the reference ``Single`` role train;
* the reference print lines come out of ``Trainer.train`` on the GPU path.
"""
import pytest
import torch

from ddl_amd.config import TrainConfig
from ddl_amd.parallel.comm import DistEnv
from ddl_amd.parallel.roles import Trainer
from ddl_amd.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def data():
    return synthetic_mnist(n_train=3000, n_test=600, seed=11)


def _trainer(data, **kw):
    base = dict(mode="sync", shard="contiguous", batch_size=100, eval_every=0, engine="hip",
                quiet=True)
    base.update(kw)
    return Trainer(TrainConfig(**base), DistEnv(0, 1, 0, DEV), dataset=data)


def test_checkpoint_resume_continues_exactly(tmp_path, data):
    ref = _trainer(data, steps=12)
    for i in range(12):
        ref.train_step(i)
    torch.cuda.synchronize()

    a = _trainer(data, steps=12)
    for i in range(6):
        a.train_step(i)
    torch.cuda.synchronize()
    from ddl_amd.utils import checkpoint as ckpt
    ckpt.save(a, str(tmp_path))
    b = _trainer(data, steps=12)
    ckpt.load(b, str(tmp_path))
    assert b.global_step == 6
    for i in range(6, 12):
        b.train_step(i)
    torch.cuda.synchronize()
    assert torch.equal(b.params, ref.params)
    for p in ref.servers:
        assert b.servers[p].t == ref.servers[p].t == 12
        assert torch.equal(b.servers[p].m, ref.servers[p].m)
        assert torch.equal(b.servers[p].v, ref.servers[p].v)


def test_async_single_gpu_matches_sync(data):
    """W = 1: the async PS (whole-shard local updates on the PS stream) applies exactly the
    updates of the sync PS, so both reach the same accuracy; and they learn."""
    tr = _trainer(data, mode="async", steps=60, lr=1e-3)
    acc0 = tr.evaluate()
    s = tr.train()
    assert s["steps"] == 60
    assert all(ps.t == 60 for ps in tr.servers.values())
    sy = _trainer(data, mode="sync", steps=60, lr=1e-3).train()
    assert abs(s["final_acc"] - sy["final_acc"]) < 0.02
    assert s["final_acc"] > max(0.5, acc0 + 0.2)


def test_single_role_on_gpu_prints_reference_lines(capsys, data):
    cfg = TrainConfig(mode="single", shard="none", steps=20, eval_every=10, engine="hip")
    tr = Trainer(cfg, DistEnv(0, 1, 0, DEV), dataset=data)
    tr.train()
    out = capsys.readouterr().out
    assert "epoch: 0 batch: 0 accuracy:" in out
    assert "epoch: 0 batch: 10 accuracy:" in out
    assert "final accuracy:" in out and "Time:" in out


def test_async_eval_reports_the_same_accuracies(data):
    """Periodic eval on the side stream from parameter snapshots (parallel/async_eval.py)
    scores exactly the parameters after each eval step: same accuracy sequence as the in-line
    eval, reported in order, with a time to target."""
    hist = []
    for eval_async in (False, True):
        tr = _trainer(data, shard="flat", steps=30, eval_every=5, eval_async=eval_async,
                      target_acc=0.0, lr=1e-3)
        s = tr.train()
        hist.append([(h["step"], h["acc"]) for h in tr.history])
        assert s["time_to_target"] is not None and s["time_to_target"] > 0
        walls = [h["wall"] for h in tr.history]
        assert walls == sorted(walls)
    assert len(hist[0]) == 6
    assert hist[0] == hist[1]


def test_async_local_elision_matches_inbox_copy(data, monkeypatch):
    """W = 1 async over xGMI (3 PS, one worker: the arrival order is fixed): the local push
    elision on and off (the apply reads the gradient in place / from the inbox) apply the same
    Adam steps in the same order, so 12-step runs are bit-identical.  (The service path: at W = 1
    the default is the runner's in-line applies, tests/test_xgmi_gpu.py.)"""
    monkeypatch.setenv("DDL_ASYNC_INLINE", "0")
    runs = []
    for elide in ("1", "0"):
        monkeypatch.setenv("DDL_ASYNC_ELIDE_LOCAL", elide)
        tr = _trainer(data, mode="async", shard="flat", steps=12, exchange_backend="xgmi")
        s = tr.train()
        assert tr.exchange.service_mode == "host"
        assert s["steps"] == 12 and all(ps.t == 12 for ps in tr.servers.values())
        torch.cuda.synchronize()
        runs.append(tr.params.clone())
    assert torch.equal(runs[0], runs[1])


def test_async_xgmi_push_tails_match_push_kernels(data, monkeypatch):
    """W = 1 async over the xGMI data plane (segment-aligned flat plan: 3 PS): the gradient
    pushes riding as tail blocks of the next segment's launch (default) and the stand-alone
    push kernels deliver the same bytes, and the GPU-side pull gate (default) orders the next
    forward after the round exactly like the host wait, so 12-step runs are bit-identical.  One step of the
    async plane equals one local (sync-path) step to rounding: the update is the same Adam in a
    different kernel (FMA contraction may differ by an ulp; over later steps Adam's early
    sign-normalised updates and the ReLU / max-pool switches amplify that into ~1e-4 parameter
    differences, scripts/async_parity_probe.py, so only the first step is compared).  The push /
    board / apply / gate chain: DDL_ASYNC_INLINE=0 (the W = 1 default applies in line)."""
    monkeypatch.setenv("DDL_ASYNC_INLINE", "0")
    runs = []
    for tail, gate in ((True, True), (False, True), (True, False)):
        tr = _trainer(data, mode="async", shard="flat", steps=12, exchange_backend="xgmi")
        assert tr.num_ps == 3 and tr.exchange.runner is not None
        tr.exchange.runner.set_use_tail(tail)
        tr.exchange.runner.set_gate(gate)
        s = tr.train()
        assert s["steps"] == 12 and all(ps.t == 12 for ps in tr.servers.values())
        torch.cuda.synchronize()
        runs.append(tr)
    assert torch.equal(runs[0].params, runs[1].params)
    assert torch.equal(runs[0].params, runs[2].params)
    one = _trainer(data, mode="async", shard="flat", steps=1, exchange_backend="xgmi")
    one.train()
    loc = _trainer(data, mode="async", shard="flat", steps=1)  # W = 1 local: the sync step
    assert loc.async_as_sync
    loc.train()
    torch.cuda.synchronize()
    for t in range(14):
        lo, hi = one.plan.tensor_extent(t)
        lo2, hi2 = loc.plan.tensor_extent(t)
        torch.testing.assert_close(one.params[lo:hi], loc.params[lo2:hi2], rtol=1e-6, atol=1e-7)
