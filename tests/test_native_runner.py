"""The C++ SyncRunner (csrc/kernels/runner.hip) vs the Python SyncExchange on one GPU.

Both enqueue the same HIP kernels on the same plan ranges, so after several steps the
parameters, the Adam moments and the PS step counters must be bit-identical — for every
shard policy (units with one / several PS, several ranges per unit, bucketed flat plan),
with and without overlap, for Adam and momentum.
"""
import pytest
import torch

from ddl_amd.config import TrainConfig
from ddl_amd.parallel.comm import DistEnv
from ddl_amd.parallel.roles import Trainer
from ddl_amd.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data():
    return synthetic_mnist(n_train=2000, n_test=500, seed=5)


def _run(data, native, steps=6, ready=None, sched=None, **kw):
    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", steps=steps, batch_size=100, eval_every=0, engine="hip",
                      quiet=True, native_exchange=native, **kw)
    tr = Trainer(cfg, env, dataset=data)
    if sched is not None:  # {op: (tile config, split)} overrides of the engine defaults
        e = tr.engine.eng
        cf, sp = e.get_cfg(), e.get_splits()
        for op, (c, s_) in sched.items():
            cf[op], sp[op] = c, s_
        e.set_cfg(cf)
        e.set_splits(sp)
    if ready is not None:
        tr.exchange.runner.set_ready_flags(ready)
    assert getattr(tr.exchange, "native", False) == native
    if kw.get("force_collectives"):
        if kw.get("exchange_backend") == "xgmi":
            assert tr.exchange.peer is not None
        else:
            assert tr.exchange.runner.has_comm()
        assert any(u.kind != "local" for u in tr.exchange.units)
    for i in range(steps):
        tr.train_step(i)
    torch.cuda.synchronize()
    sync = getattr(tr.exchange, "sync_ps_state", None)  # replicated last-bucket state -> PS
    if sync is not None:
        sync()
    state = {p: (s.t, s.m.clone(), None if s.v is None else s.v.clone())
             for p, s in tr.servers.items()}
    return tr.params.clone(), state


@pytest.mark.parametrize("kw", [
    dict(shard="contiguous"),
    dict(shard="greedy", num_ps=3),
    dict(shard="contiguous", num_ps=2, overlap=False),
    dict(shard="flat"),
    dict(shard="lpt", num_ps=4, optimizer="momentum"),
    dict(shard="contiguous", optimizer="sgd"),   # the momentum kernel with mu = 0, natively
])
def test_native_matches_python_exchange(data, kw):
    p_py, s_py = _run(data, False, **kw)
    p_nat, s_nat = _run(data, True, **kw)
    assert torch.equal(p_py, p_nat)
    assert s_py.keys() == s_nat.keys()
    for p in s_py:
        assert s_py[p][0] == s_nat[p][0]
        assert torch.equal(s_py[p][1], s_nat[p][1])
        if s_py[p][2] is not None:
            assert torch.equal(s_py[p][2], s_nat[p][2])


def test_fc2_reduce_in_head_is_bit_identical(data, monkeypatch):
    """With fc2's forward on a split-K tile, the native step leaves its reduce to the head
    kernel (engine.hip Engine::forward defer_fc2, head.hip head_fused_fc2_kernel: same summation
    order as the wide reduce launch).  Parameters and Adam state match the separate-launch step
    bitwise."""
    # fc2's forward on the split-K 32x32 tile (config 3, split 16): the default runs it on the
    # 16-row K-wave launch (CFG_KW16), whose epilogue writes h2 itself
    sched = {5: (3, 16)}
    monkeypatch.setenv("DDL_FC2_REDUCE_IN_HEAD", "0")
    p_sep, s_sep = _run(data, True, sched=sched, shard="flat")
    monkeypatch.setenv("DDL_FC2_REDUCE_IN_HEAD", "1")
    p_head, s_head = _run(data, True, sched=sched, shard="flat")
    assert torch.equal(p_sep, p_head)
    for p in s_sep:
        assert torch.equal(s_sep[p][1], s_head[p][1])


def test_native_runner_trains(data):
    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", shard="contiguous", steps=60, batch_size=100, eval_every=0,
                      engine="hip", quiet=True, lr=1e-3)
    tr = Trainer(cfg, env, dataset=data)
    acc0 = tr.evaluate()
    for i in range(60):
        tr.train_step(i)
    assert tr.evaluate() > max(0.5, acc0 + 0.2)


@pytest.mark.parametrize("kw", [
    dict(shard="flat"),                       # RS unit -> ncclReduceScatter/AllGather
    dict(shard="contiguous"),                 # REDUCE units -> grouped ncclReduce/Broadcast
    dict(shard="greedy", num_ps=3),           # several PS hosts, several ranges per unit
    dict(shard="contiguous", num_ps=2, overlap=False),
    dict(shard="flat", exchange_backend="xgmi"),  # fused xGMI bucket kernels, push to self
    dict(shard="flat", exchange_backend="xgmi", overlap=False),
    dict(shard="flat", exchange_backend="xgmi", optimizer="sgd"),
    dict(shard="flat", exchange_backend="xgmi", optimizer="momentum"),
    # tensor-granular plans on xGMI OWNER buckets (one push / owner update / pull kernel per
    # unit; at W = 1 every unit is owned here): reference none / contiguous / greedy
    dict(shard="none", exchange_backend="xgmi"),
    dict(shard="contiguous", exchange_backend="xgmi"),
    dict(shard="greedy", num_ps=3, exchange_backend="xgmi"),
    dict(shard="lpt", num_ps=4, exchange_backend="xgmi", optimizer="momentum"),
])
def test_forced_collectives_on_one_rank_match_local(data, kw):
    """The multi-GPU exchange path on one GPU: torch's librccl resolved by dlsym, a 1-rank
    communicator, the comm stream waiting on per-segment events, RS/AG and grouped
    reduce/broadcast units.  With one rank every collective is a copy, so the result must be
    bit-identical to the local-update path."""
    p_loc, s_loc = _run(data, True, **kw)
    p_col, s_col = _run(data, True, force_collectives=True, **kw)
    assert torch.equal(p_loc, p_col)
    for p in s_loc:
        assert s_loc[p][0] == s_col[p][0]
        assert torch.equal(s_loc[p][1], s_col[p][1])
        if s_loc[p][2] is not None:
            assert torch.equal(s_loc[p][2], s_col[p][2])


@pytest.mark.parametrize("shard", ["flat", "contiguous"])
def test_last_segment_exchange_stream_placement(data, shard, monkeypatch):
    """The last backward segment's collectives on the compute stream (default) or on the comm
    stream behind an event (DDL_LAST_ON_MAIN=0): same kernels in the same RCCL order, so the
    results are bit-identical."""
    monkeypatch.setenv("DDL_LAST_ON_MAIN", "1")
    p_main, s_main = _run(data, True, force_collectives=True, shard=shard)
    monkeypatch.setenv("DDL_LAST_ON_MAIN", "0")
    p_comm, s_comm = _run(data, True, force_collectives=True, shard=shard)
    assert torch.equal(p_main, p_comm)
    for p in s_main:
        assert torch.equal(s_main[p][1], s_comm[p][1])
        assert torch.equal(s_main[p][2], s_comm[p][2])


def test_rccl_probe_resolves_torch_librccl():
    from ddl_amd.ops import native
    assert native.ops().SyncRunner.probe() == ""


@pytest.mark.parametrize("shard", ["flat", "contiguous"])
def test_optimizer_tail_matches_end_of_step_update(data, shard):
    """W = 1: segment s's Adam riding as extra blocks of segment s+1's dual GEMM launch
    (csrc/kernels/tail.h), and the last segment's Adam inside conv1's weight-gradient reduce
    launch (conv1's in the reduce epilogue, conv2's as tail blocks: gemm.h
    splitk_wide_reduce_tail), give bit-identical parameters and moments to one coalesced Adam
    launch after the backward."""
    out = []
    # (tail, last segment's update inside conv1's weight-gradient reduce launch)
    for tail, final in ((True, True), (True, False), (False, False)):
        env = DistEnv(0, 1, 0, torch.device("cuda", 0))
        cfg = TrainConfig(mode="sync", shard=shard, steps=5, batch_size=100, eval_every=0,
                          engine="hip", quiet=True)
        tr = Trainer(cfg, env, dataset=data)
        tr.exchange.runner.set_use_tail(tail)
        tr.exchange.runner.set_final_in_reduce(final)
        for i in range(5):
            tr.train_step(i)
        torch.cuda.synchronize()
        s = tr.servers[0]
        out.append((tr.params.clone(), s.m.clone(), s.v.clone()))
    for ref in out[1:]:
        for a, b in zip(out[0], ref):
            assert torch.equal(a, b)


def _train_async(data, **kw):
    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="async", steps=6, batch_size=100, eval_every=0, engine="hip",
                      quiet=True, shard="contiguous", **kw)
    tr = Trainer(cfg, env, dataset=data)
    tr.train()
    torch.cuda.synchronize()
    return tr


def test_rccl_async_self_sessions_match_local(data):
    """The async RCCL data plane (csrc/kernels/rccl_async.hip) on one GPU: with one rank every
    push / pull is an RCCL send/recv to itself inside a session (comm thread, comm stream, PS
    apply on its private copy), bit-equal to the local async step; provenance verified."""
    from ddl_amd.parallel.async_rccl import RcclAsyncExchange
    loc = _train_async(data)
    assert loc.async_as_sync
    rc = _train_async(data, exchange_backend="rccl", check_provenance=True)
    assert isinstance(rc.exchange, RcclAsyncExchange)
    assert torch.equal(loc.params, rc.params)
    assert rc.servers[0].t == loc.servers[0].t == 6


@pytest.mark.parametrize("backend", ["rccl", "xgmi"])
def test_async_resume_continues_exactly(tmp_path, data, backend):
    """an async job (RCCL sessions / xGMI data plane, W = 1) checkpointed at
    step 3 and resumed continues exactly: the native PS picks up the restored step counter
    (RcclAsync.set_t / AsyncService built in start()), so parameters and t equal the
    uninterrupted 6-step run's."""
    full = _train_async(data, exchange_backend=backend)
    ck = str(tmp_path / "ck")
    part = _train_async(data, exchange_backend=backend, checkpoint_dir=ck, checkpoint_every=3,
                        max_steps=3)
    assert part.global_step == 3
    res = _train_async(data, exchange_backend=backend, checkpoint_dir=ck, resume=True)
    assert res.global_step == 6
    assert all(s.t == 6 for s in res.servers.values())
    assert all(s.t == f.t for s, f in zip(res.servers.values(), full.servers.values()))
    assert torch.equal(res.params, full.params)


@pytest.mark.parametrize("backend", ["rccl", "xgmi"])
def test_ready_flag_handoff_matches_events(data, backend):
    """The comm stream's hand-off: READY flags for every segment (default), only after the first
    segment, events, and — on a HIGH-priority compute stream, where a gate could share the comm
    stream's hardware queue — the automatic fallback to events.  Same kernels in the same order
    on both streams, so all four are bit-identical."""
    kw = dict(shard="flat", force_collectives=True, exchange_backend=backend)
    ref = _run(data, True, **kw)
    runs = [_run(data, True, ready=1, **kw), _run(data, True, ready=0, **kw)]
    with torch.cuda.stream(torch.cuda.Stream(priority=-1)):
        runs.append(_run(data, True, **kw))
    torch.cuda.synchronize()
    for p, st in runs:
        assert torch.equal(ref[0], p)
        for q in ref[1]:
            assert torch.equal(ref[1][q][1], st[q][1])


@pytest.mark.parametrize("kw", [dict(shard="flat"), dict(shard="contiguous"),
                                dict(shard="flat", exchange_backend="xgmi"),
                                dict(shard="greedy", num_ps=3, exchange_backend="xgmi")])
def test_handoff_check_proves_ready_flags(data, kw):
    """the forced 1-rank rehearsal runs the bench's hand-off check — K steps
    with the event hand-off and K with the READY flags from the same state, bit-identical —
    keeps the flags, and leaves the trainer's state exactly as before the check."""
    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", steps=20, batch_size=100, eval_every=0, engine="hip",
                      quiet=True, force_collectives=True, **kw)
    tr = Trainer(cfg, env, dataset=data)
    before = tr.params.clone()
    t_before = {p: s.t for p, s in tr.servers.items()}
    res = tr.exchange.handoff_check(tr, steps=4)
    assert res["handoff"] == "ready_flags", res
    assert res["modes_bit_identical"] and res["ranks_bit_identical"]
    assert torch.equal(tr.params, before)
    assert {p: s.t for p, s in tr.servers.items()} == t_before
    # and training continues from the restored state exactly like a fresh trainer
    for i in range(3):
        tr.train_step(i)
    torch.cuda.synchronize()
    p_fresh, _ = _run(data, True, steps=3, force_collectives=True, **kw)
    assert torch.equal(tr.params, p_fresh)
