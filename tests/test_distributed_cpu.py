"""Protocol tests on CPU with the gloo backend (the fake backend for a GPU-less box,
SURVEY.md §4): the same Trainer / exchange code that runs over RCCL on MI355X, run as
W processes; synchronous results must equal a single-process simulation of the
parameter-server math, asynchronous runs must finish with every push served."""
import os

import pytest
import torch

from dist_helpers import spawn, train_rank, simulate_sync
from conftest import free_port

pytestmark = pytest.mark.slow

BASE = dict(mode="sync", steps=3, batch_size=50, eval_every=0, quiet=True, engine="torch",
            data="synthetic", watchdog_s=120.0)


def _run(tmp_path, world, **kw):
    cfg = dict(BASE, **kw)
    spawn(train_rank, world, free_port(), cfg, str(tmp_path))
    return [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=False) for r in range(world)], cfg


def _canon(rec):
    """plan-ordered params -> canonical v0..v13 order"""
    from ddl_amd.models.layout import TENSORS
    p, off = rec["params"], rec["plan_offsets"]
    return torch.cat([p[off[t.index]:off[t.index] + t.numel] for t in TENSORS])


@pytest.mark.parametrize("world,kw", [
    (2, dict(shard="contiguous")),                 # mnist_sync_sharding
    (3, dict(shard="greedy")),                     # mnist_sync_sharding_greedy
    (2, dict(shard="none")),                       # mnist_sync (1 PS)
    (2, dict(shard="flat")),                       # RS/AG fast path
    (4, dict(shard="flat", data_sharding="stride")),  # the bench configuration at W = 4
    (3, dict(shard="lpt")),
    (3, dict(shard="contiguous", num_ps=2)),       # fewer PS than workers
    (2, dict(shard="contiguous", num_ps=5)),       # several PS per process
    (2, dict(shard="contiguous", grad_reduce="mean")),
    (2, dict(shard="contiguous", data_sharding="stride")),
])
def test_sync_matches_single_process_simulation(tmp_path, world, kw):
    recs, cfg = _run(tmp_path, world, **kw)
    ref = simulate_sync(cfg, world)
    for r, rec in enumerate(recs):
        got = _canon(rec)
        # fp32 sums of W gradients in a different order; Adam can move a ~0 gradient by
        # up to lr per step, so allow 2e-5 (lr * steps = 3e-4)
        assert torch.allclose(got, ref, atol=2e-5, rtol=0), (r, float((got - ref).abs().max()))
    # every worker ends with identical parameters
    for rec in recs[1:]:
        assert torch.equal(_canon(rec), _canon(recs[0]))


@pytest.mark.parametrize("world,shard", [(3, "contiguous"), (2, "none"), (3, "greedy")])
def test_reference_quirks_reproduced(tmp_path, world, shard):
    """--ref-quirks: Q1 (the single sync PS adds worker 1's buffer to itself: 2 g_1 + g_2 + ...),
    Q2 (the sharded sync PS aliases one receive buffer: g_last * 2**(W-1)) and Q4 (independent
    init per process; the PS starts from its host's init, step-0 gradients from each worker's
    own) against the single-process simulation of exactly that math."""
    recs, cfg = _run(tmp_path, world, shard=shard, ref_quirks=True)
    ref = simulate_sync(cfg, world)
    for r, rec in enumerate(recs):
        got = _canon(rec)
        assert torch.allclose(got, ref, atol=2e-5, rtol=0), (r, float((got - ref).abs().max()))
    # after the first pull every worker holds the PS parameters
    for rec in recs[1:]:
        assert torch.equal(_canon(rec), _canon(recs[0]))


# ---- W = 8: every reference variant at the size of BASELINE configs 3-5 (8 workers) --------
W8 = dict(steps=2, batch_size=10)


@pytest.mark.parametrize("kw", [
    dict(shard="none"),                            # mnist_sync (1 PS on rank 0, 8 workers)
    dict(shard="contiguous"),                      # mnist_sync_sharding, P = 8 (4.76x imbalance)
    dict(shard="greedy"),                          # mnist_sync_sharding_greedy, P = 8
    dict(shard="flat", data_sharding="stride"),    # the bench plan: RS / AG per bucket
    dict(shard="contiguous", num_ps=3),            # run.sh 3 8: fewer PS than workers
    dict(shard="contiguous", num_ps=11),           # run.sh 11 8: PS 8..10 on ranks 0..2
])
def test_sync_w8_matches_simulation(tmp_path, kw):
    recs, cfg = _run(tmp_path, 8, **W8, **kw)
    ref = simulate_sync(cfg, 8)
    for r, rec in enumerate(recs):
        got = _canon(rec)
        assert torch.allclose(got, ref, atol=2e-5, rtol=0), (r, float((got - ref).abs().max()))
    for rec in recs[1:]:
        assert torch.equal(_canon(rec), _canon(recs[0]))


@pytest.mark.parametrize("kw", [dict(shard="contiguous"), dict(shard="greedy"),
                                dict(shard="none")])
def test_async_w8_provenance(tmp_path, kw):
    """mnist_async_sharding / _greedy / mnist_async at W = 8: every push served once, in
    order, with its bytes checksummed at the PS; each PS counts W x steps updates."""
    recs, cfg = _run(tmp_path, 8, mode="async", check_provenance=True, **W8, **kw)
    from ddl_amd.parallel.sharding import make_plan
    num_ps = 1 if kw["shard"] == "none" else 8
    plan = make_plan(kw["shard"], num_ps)
    ps_t = {}
    for r, rec in enumerate(recs):
        ps_t.update(rec["ps_t"])
        hosted = sum(1 for p in range(plan.num_ps) if plan.host_rank(p, 8) == r)
        assert len(rec["provenance"]) == hosted * 7 * cfg["steps"]
        assert torch.isfinite(rec["params"]).all()
    assert sorted(ps_t) == list(range(num_ps))
    assert all(t == 8 * cfg["steps"] for t in ps_t.values()), ps_t


@pytest.mark.parametrize("world,shard", [(3, "greedy"), (2, "none"), (3, "contiguous")])
def test_async_serves_every_push(tmp_path, world, shard):
    recs, cfg = _run(tmp_path, world, mode="async", shard=shard)
    steps = cfg["steps"]
    num_ps = 1 if shard == "none" else world
    ps_t = {}
    for rec in recs:
        ps_t.update(rec["ps_t"])
    # each PS applied exactly one Adam step per push from every worker (Q9 semantics)
    assert sorted(ps_t) == list(range(num_ps))
    assert all(t == world * steps for t in ps_t.values()), ps_t
    for rec in recs:
        assert torch.isfinite(rec["params"]).all()


@pytest.mark.parametrize("world,num_ps", [(2, 4), (3, 9)])
def test_async_segment_aligned_flat_plan(tmp_path, world, num_ps):
    """The async flat plan with the HIP engine's backward segments (segment-aligned: every PS
    range inside one group, the tiny fc3 segment folded into the next, sharding.async_groups;
    P the smallest balanced multiple of W): W = 2 -> 4 PS, W = 3 -> 9, uneven ranges — every
    push served once in order with checksummed bytes, each PS at W x steps."""
    from ddl_amd.models import HIP_SEGMENTS
    recs, cfg = _run(tmp_path, world, mode="async", shard="flat", check_provenance=True,
                     _segments=HIP_SEGMENTS)
    ps_t = {}
    for r, rec in enumerate(recs):
        assert rec["num_ps"] == num_ps
        ps_t.update(rec["ps_t"])
        assert len(rec["provenance"]) == (num_ps // world) * (world - 1) * cfg["steps"]
        assert torch.isfinite(rec["params"]).all()
    assert sorted(ps_t) == list(range(num_ps))
    assert all(t == world * cfg["steps"] for t in ps_t.values()), ps_t


@pytest.mark.parametrize("world,kw", [(3, dict(shard="greedy")), (3, dict(shard="contiguous",
                                                                          num_ps=2))])
def test_async_provenance_checked(tmp_path, world, kw):
    """Race-detection mode: every remote push is checksummed and its
    (worker, step) order verified at the PS (train() raises otherwise); the log holds one
    entry per applied remote push."""
    recs, cfg = _run(tmp_path, world, mode="async", check_provenance=True, **kw)
    steps = cfg["steps"]
    from ddl_amd.parallel.sharding import make_plan
    plan = make_plan(kw["shard"], kw.get("num_ps", world))
    for r, rec in enumerate(recs):
        hosted = sum(1 for p in range(plan.num_ps) if plan.host_rank(p, world) == r)
        prov = rec["provenance"]
        assert len(prov) == hosted * (world - 1) * steps
        assert all(w != r for (w, _, _, _) in prov)


def test_async_single_worker_equals_sync(tmp_path):
    """W=1: async and sync PS do the same math."""
    a, cfg = _run(tmp_path, 1, mode="async", shard="contiguous")
    ref = simulate_sync(dict(cfg, mode="sync"), 1)
    assert torch.allclose(_canon(a[0]), ref, atol=2e-6, rtol=0)


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_eval_equals_full_eval(tmp_path, world):
    """Sync mode scores 1/W of the test set per rank (odd split: 301 images) and
    all-reduces the counts: same accuracy as every rank scoring the whole set."""
    from dist_helpers import eval_rank, spawn
    spawn(eval_rank, world, free_port(), str(tmp_path))
    res = [torch.load(tmp_path / f"eval{r}.pt") for r in range(world)]
    for r in res:
        assert r["dist"] == r["full"] == res[0]["full"]


@pytest.mark.parametrize("case", ["agree", "flags_diverge", "replicas_diverge"])
def test_handoff_vote_refuses_diverged_replicas(tmp_path, case):
    """The READY-flag hand-off check's collective verdict (native_exchange.handoff_vote) over
    gloo, W = 2: every rank agreeing keeps the flags; a rank whose READY-flag run alone differs
    sends every rank back to the event hand-off; a rank whose replica differs under the event
    hand-off too makes EVERY rank refuse the data plane (NativeUnavailable) instead of training
    on diverged replicas."""
    from dist_helpers import handoff_vote_rank
    world = 2
    spawn(handoff_vote_rank, world, free_port(), str(tmp_path), case)
    outs = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=False)
            for r in range(world)]
    if case == "agree":
        assert all(o["ok"] and o["ranks_agree"] and o["modes_agree"] for o in outs)
    elif case == "flags_diverge":
        assert all(not o["ok"] and "refused" not in o for o in outs)
    else:
        assert all("refused" in o and "diverge" in o["refused"] for o in outs)
