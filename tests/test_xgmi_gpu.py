"""The xGMI peer-memory exchange (csrc/kernels/xgmi.hip) as a real multi-process job.

W worker processes share ONE GPU (default process group over gloo, ``DDL_DIST_BACKEND``):
RCCL refuses two ranks on one device, but the xGMI exchange only needs IPC-mapped memory, so
the whole W > 1 native step — IPC handle exchange, self-test vote, per-bucket push / owner
Adam / pull kernels on the comm stream, the final wait on the compute stream, cross-process
flag epochs — runs here exactly as on an 8-GPU node (where the same stores cross xGMI links).

The parameters after K steps must be BIT-identical on every rank and equal to a one-process
simulation of the PS math with the same HIP engine: each rank's gradient on its own batch and
dropout seed, summed in rank order (the kernel's order), one TF1 Adam step per global step.
"""
import os
import sys
import traceback

import pytest
import torch

from conftest import ROOT, free_port

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

STEPS = 4


def _canon(params, offsets):
    from ddl_amd.models.layout import TENSORS
    return torch.cat([params[offsets[t.index]:offsets[t.index] + t.numel] for t in TENSORS])


# Eight processes on ONE card: each pinned to one hardware queue (GPU_MAX_HW_QUEUES=1, HIP
# reads it at init), so the box runs 8 queues, not 8 x 4 (the oversubscribed regime round 2's
# W = 8 runs stalled in), and with the inbox checksums on (DDL_XGMI_CHECK=1: every owner
# verifies every pushed slice against its pusher's checksum, error code 3 on a mismatch).
W8_ENV = dict(GPU_MAX_HW_QUEUES="1", DDL_XGMI_CHECK="1", DDL_XGMI_TIMEOUT_S="60")
# W = 8 on one card runs with EXACTLY eight GPU processes: rank 0 is this pytest process
# (which already holds a GPU context from the earlier tests) and ranks 1..7 are spawned.  The
# round-3 abort (HSA_STATUS_ERROR_ILLEGAL_INSTRUCTION in a GEMM dual kernel,
# profiles/r3_w8_one_gpu_fault.log) happened with mp.spawn's eight ranks PLUS this process — nine
# processes with hardware queues, one more than the eight compute VMIDs the kernel driver's
# scheduler keeps resident at once, so the run list was over-subscribed and the scheduler
# time-sliced whole processes by preempting their waves (context save / restore) — the regime
# every W = 8 stall, divergence and abort on one card was seen in, and one no 8-GPU node (one
# process per GPU) ever enters.  docs/DESIGN.md "W = 8 on one card: the cause".
def _inproc_rank0(fn, world, *args):
    """fn(rank, world, *args) on ranks 1..world-1 in spawned processes and rank 0 here."""
    import gc
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    kids = [ctx.Process(target=fn, args=(r, world, *args)) for r in range(1, world)]
    for k in kids:
        k.start()
    saved = dict(os.environ)
    ok = False
    try:
        fn(0, world, *args)
        ok = True
    finally:
        os.environ.clear()
        os.environ.update(saved)
        for k in kids:
            k.join(timeout=180 if ok else 5)
            if k.is_alive():
                k.kill()
                k.join()
        gc.collect()
        torch.cuda.synchronize()
    assert all(k.exitcode == 0 for k in kids), [k.exitcode for k in kids]


def _rank(rank, world, port, outdir, kw):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    kw = dict(kw)
    extra_env = kw.pop("_env", {})
    kw.pop("_ps", None)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DDL_DIST_BACKEND="gloo",
                      DDL_XGMI_TIMEOUT_S="20")
    os.environ.update(extra_env)
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed()
        assert env.device.index == 0
        shard = kw.pop("shard", "flat")
        cfg = TrainConfig(mode="sync", shard=shard, steps=STEPS, batch_size=100, eval_every=0,
                          engine="hip", quiet=True, data_sharding="stride",
                          exchange_backend="xgmi", **kw)
        tr = Trainer(cfg, env, dataset=synthetic_mnist(2000, 500, seed=5))
        ex = tr.exchange
        assert getattr(ex, "native", False) and ex.peer is not None, "xgmi path not taken"
        # tensor-granular plans: one xGMI OWNER bucket per exchange unit, hosted where its PS is
        owner = shard != "flat" or tr.plan.num_ps != world
        assert all((ex.peer.owner(b) >= 0) == owner for b in range(len(ex.peer.nslices()))), \
            "wrong xGMI bucket kind for the plan"
        sums = []
        for i in range(STEPS):
            tr.train_step(i)
            sums.append(_canon(tr.params, tr.plan.tensor_offsets).double().sum().item())
        torch.cuda.synchronize()
        ex.check()
        acc = tr.evaluate()
        torch.save({"params": _canon(tr.params, tr.plan.tensor_offsets).cpu(), "acc": acc,
                    "sums": sums,
                    "t": {p: s.t for p, s in tr.servers.items()}},
                   os.path.join(outdir, f"rank{rank}.pt"))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


def _simulate(world, kw):
    from ddl_amd.models import engine_segments
    from ddl_amd.models.hip_engine import HipEngine
    from ddl_amd.models.mnist_cnn import init_params_
    from ddl_amd.ops import native, rng
    from ddl_amd.ops.adam import AdamHyper, adam_coeffs
    from ddl_amd.parallel.sharding import make_plan
    from ddl_amd.utils.data import synthetic_mnist, batch_indices
    dev = torch.device("cuda", 0)
    data = synthetic_mnist(2000, 500, seed=5).to(dev)
    plan = make_plan("flat", world, buckets=engine_segments("hip", dev))
    params = torch.zeros(plan.total, device=dev)
    init_params_(params, plan.tensor_offsets, 0)
    grads = torch.zeros_like(params)
    acc, m, v = torch.zeros_like(params), torch.zeros_like(params), torch.zeros_like(params)
    eng = HipEngine(params, grads, plan.tensor_offsets, batch=100, graph=False)
    h = AdamHyper()
    coef = kw.get("coef", [1.0] * world)
    sums = []
    for step in range(STEPS):
        acc.zero_()
        for r in range(world):
            lo, hi = batch_indices(step, 100, data.total_batch, r, world, "stride")
            eng.forward_backward(data.x_train[lo:hi], data.y_train[lo:hi], 0.5,
                                 rng.step_seed(0, r, step))
            acc.add_(grads * coef[r] if coef[r] != 1.0 else grads)
        scale = 1.0 / world if kw.get("grad_reduce") == "mean" else 1.0
        native.ops().adam_flat(params, acc, m, v, adam_coeffs(h, step + 1), h.beta1, h.beta2,
                               h.eps, scale)
        sums.append(_canon(params, plan.tensor_offsets).double().sum().item())
    torch.cuda.synchronize()
    return _canon(params, plan.tensor_offsets).cpu(), sums


@pytest.mark.parametrize("world,kw", [
    (2, {}),
    (3, dict(grad_reduce="mean")),
    (4, dict(overlap=False)),
    (2, dict(_env=dict(DDL_REPL_LAST="0"))),     # last bucket by its chunk owners
    (4, dict(_env=dict(DDL_XGMI_CHECK="1"))),
    pytest.param(8, dict(_env=W8_ENV), id="w8"),  # the 8-worker size of BASELINE configs 3-5
    # tensor-granular plans on owner buckets (every rank pushes a unit to the rank hosting its
    # PS, which sums, updates and pushes the parameters back):
    pytest.param(2, dict(shard="none"), id="2-none"),              # BASELINE config 2: 1 PS + 2
    pytest.param(2, dict(shard="contiguous"), id="2-contig"),      # mnist_sync_sharding
    pytest.param(4, dict(shard="contiguous"), id="4-contig"),
    pytest.param(3, dict(shard="contiguous", num_ps=5), id="3-contig-5ps"),  # 2 PS on some hosts
    pytest.param(4, dict(shard="greedy", grad_reduce="mean"), id="4-greedy"),
    pytest.param(8, dict(shard="contiguous", _env=W8_ENV), id="w8-contig"),  # BASELINE config 3
    pytest.param(8, dict(shard="greedy", _env=W8_ENV), id="w8-greedy"),
])
def test_xgmi_exchange_matches_simulation(tmp_path, world, kw):
    import torch.multiprocessing as mp
    if world == 8:
        _inproc_rank0(_rank, world, free_port(), str(tmp_path), kw)
    else:
        mp.spawn(_rank, args=(world, free_port(), str(tmp_path), kw), nprocs=world, join=True)
    recs = [torch.load(os.path.join(tmp_path, f"rank{r}.pt")) for r in range(world)]
    for rec in recs[1:]:
        assert torch.equal(rec["params"], recs[0]["params"])
        assert rec["acc"] == recs[0]["acc"]
    assert all(t == STEPS for rec in recs for t in rec["t"].values())
    ref, ref_sums = _simulate(world, {k: v for k, v in kw.items()
                                      if k not in ("overlap", "_env", "shard", "num_ps")})
    got = recs[0]["params"]
    diff = float((got - ref).abs().max())
    # per-step parameter checksums localise a divergence (which step, which rank)
    steps = [[rec["sums"][i] for rec in recs] for i in range(STEPS)]
    assert torch.equal(got, ref), f"max |diff| {diff}; per-step sums {steps} vs {ref_sums}"


def _handoff_rank(rank, world, port, outdir, perturb):
    """One-card W = 2 xGMI sync trainer; its READY-flag hand-off check with (perturb) or without
    an injected digest disagreement on the last rank."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DDL_DIST_BACKEND="gloo",
                      DDL_XGMI_TIMEOUT_S="20")
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.native_exchange import NativeUnavailable
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed()
        cfg = TrainConfig(mode="sync", shard="flat", steps=STEPS, batch_size=100, eval_every=0,
                          engine="hip", quiet=True, data_sharding="stride",
                          exchange_backend="xgmi")
        tr = Trainer(cfg, env, dataset=synthetic_mnist(2000, 500, seed=5))
        assert tr.exchange.peer is not None, "xgmi path not taken"
        try:
            out = tr.exchange.handoff_check(tr, steps=2,
                                            _perturb_rank=world - 1 if perturb else None)
        except NativeUnavailable as e:
            out = {"refused": str(e)}
        torch.cuda.synchronize()
        torch.save(out, os.path.join(outdir, f"rank{rank}.pt"))
        dist.barrier()
        tr.exchange.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


@pytest.mark.parametrize("perturb", [False, True])
def test_handoff_check_refuses_diverged_replicas(tmp_path, perturb):
    """One card, W = 2 over xGMI: the hand-off check proves the READY flags (both ranks, same
    bits); with a digest disagreement injected on rank 1 both ranks refuse the data plane
    (NativeUnavailable) instead of falling back to events."""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_handoff_rank, args=(world, free_port(), str(tmp_path), perturb), nprocs=world,
             join=True)
    outs = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=False)
            for r in range(world)]
    if perturb:
        assert all("refused" in o and "diverge" in o["refused"] for o in outs), outs
    else:
        assert all(o["handoff"] == "ready_flags" and o["ranks_bit_identical"] for o in outs), outs


ASYNC_STEPS = 6


def _async_rank(rank, world, port, outdir, kw):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    kw = dict(kw)
    extra_env = kw.pop("_env", {})
    kw.pop("_ps", None)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DDL_DIST_BACKEND="gloo",
                      DDL_XGMI_TIMEOUT_S="20")
    os.environ.update(extra_env)
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.async_xgmi import AsyncPeerExchange
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed()
        cfg = TrainConfig(mode="async", steps=ASYNC_STEPS, batch_size=100, eval_every=0,
                          engine="hip", quiet=True, data_sharding="stride",
                          exchange_backend="xgmi", check_provenance=True, watchdog_s=120.0,
                          **kw)
        tr = Trainer(cfg, env, dataset=synthetic_mnist(2000, 500, seed=5))
        assert isinstance(tr.exchange, AsyncPeerExchange), type(tr.exchange)
        want_native = extra_env.get("DDL_ASYNC_NATIVE", "1") == "1"
        assert (tr.exchange.runner is not None) == want_native, "native async step not taken"
        s = tr.train()  # verify_provenance runs inside (check_provenance=True)
        torch.cuda.synchronize()
        if tr.servers:  # the PS service this host ran: the native host scan, or at W = 1 the
            # runner's in-line applies (async_runner.hip set_inline)
            inline = (world == 1 and want_native
                      and extra_env.get("DDL_ASYNC_INLINE", "1") == "1")
            want = "inline" if inline else "host"
            assert tr.exchange.service_mode == want, tr.exchange.service_mode
        torch.save({"params": tr.params.cpu(), "served": tr.exchange.served,
                    "ps": {p: (sv.t, sv.params.cpu()) for p, sv in tr.servers.items()},
                    "ranges": {p: tr.plan.ps_segments(p)[0] for p in tr.servers},
                    "acc": s["final_acc"]},
                   os.path.join(outdir, f"rank{rank}.pt"))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


@pytest.mark.parametrize("world,kw", [
    (1, dict(shard="none")),                     # one worker, its own PS: in-line applies
    pytest.param(1, dict(shard="none", _env=dict(DDL_ASYNC_INLINE="0")), id="1-service"),
    (2, dict(shard="contiguous")),               # mnist_async_sharding
    (4, dict(shard="greedy", num_ps=4)),         # mnist_async_sharding_greedy
    (3, dict(shard="contiguous", num_ps=5)),     # several PS per host
    (2, dict(shard="greedy", _env=dict(DDL_ASYNC_NATIVE="0"))),  # the Python push_pull path
    # segment-aligned flat plans (sharding.async_groups + segment_aligned_num_ps): 3 PS on one
    # host, 4 on two
    pytest.param(1, dict(shard="flat", _ps=3), id="1-flat"),
    pytest.param(2, dict(shard="flat", _ps=4), id="2-flat"),

    pytest.param(8, dict(shard="contiguous", _env=dict(GPU_MAX_HW_QUEUES="1",
                                                       DDL_XGMI_TIMEOUT_S="60")), id="w8-contig"),
    pytest.param(8, dict(shard="greedy", _env=dict(GPU_MAX_HW_QUEUES="1",
                                                   DDL_XGMI_TIMEOUT_S="60")), id="w8-greedy"),
])
def test_async_xgmi_serves_every_push(tmp_path, world, kw):
    import torch.multiprocessing as mp
    if world == 8:
        _inproc_rank0(_async_rank, world, free_port(), str(tmp_path), kw)
    else:
        mp.spawn(_async_rank, args=(world, free_port(), str(tmp_path), kw), nprocs=world,
                 join=True)
    recs = [torch.load(os.path.join(tmp_path, f"rank{r}.pt")) for r in range(world)]
    n_ps = sum(len(rec["ps"]) for rec in recs)
    assert n_ps == kw.get("_ps", kw.get("num_ps", 1 if kw["shard"] == "none" else world))
    for rec in recs:
        # every hosted PS applied exactly one update per push of every worker
        for p, (t, _) in rec["ps"].items():
            assert t == world * ASYNC_STEPS, (p, t)
        assert rec["served"] == len(rec["ps"]) * world * ASYNC_STEPS
        assert torch.isfinite(rec["params"]).all()
    # the last worker a PS served holds exactly that PS's final parameters
    for rec in recs:
        for p, (_, ps_params) in rec["ps"].items():
            lo, hi = rec["ranges"][p]
            assert any(torch.equal(o["params"][lo:hi], ps_params) for o in recs), p


@pytest.mark.parametrize("shard,ps", [("none", 1), ("flat", 3)])
def test_async_inline_apply_equals_service_w1(tmp_path, shard, ps):
    """at W = 1 the pushes to the self-hosted PS are applied in-line (tail
    blocks of the next backward launch) instead of through the board, the service's apply kernel
    and the gate.  Same Adam arithmetic, same per-PS step counters, same order: the worker's
    parameters and every PS's state must be bit-identical to the service path's."""
    import torch.multiprocessing as mp
    recs = {}
    for mode in ("1", "0"):
        d = tmp_path / f"inline{mode}"
        d.mkdir()
        kw = dict(shard=shard, _ps=ps, _env=dict(DDL_ASYNC_INLINE=mode))
        mp.spawn(_async_rank, args=(1, free_port(), str(d), kw), nprocs=1, join=True)
        recs[mode] = torch.load(d / "rank0.pt")
    a, b = recs["1"], recs["0"]
    assert len(a["ps"]) == ps
    assert a["served"] == b["served"] == ps * ASYNC_STEPS
    assert torch.equal(a["params"], b["params"])
    for p in a["ps"]:
        assert a["ps"][p][0] == b["ps"][p][0] == ASYNC_STEPS
        assert torch.equal(a["ps"][p][1], b["ps"][p][1]), p
        lo, hi = a["ranges"][p]
        assert torch.equal(a["ps"][p][1], a["params"][lo:hi]), p


def _ckpt_rank(rank, world, port, outdir, kw):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DDL_DIST_BACKEND="gloo",
                      DDL_XGMI_TIMEOUT_S="20")
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed()
        cfg = TrainConfig(mode="async", steps=6, batch_size=100, eval_every=0, engine="hip",
                          quiet=True, data_sharding="stride", exchange_backend="xgmi",
                          checkpoint_dir=os.path.join(outdir, "ck"), watchdog_s=120.0, **kw)
        tr = Trainer(cfg, env, dataset=synthetic_mnist(2000, 500, seed=5))
        tr.train()  # checkpoint_every=3: a mid-run snapshot while the PS services run
        torch.save({"t": {p: s.t for p, s in tr.servers.items()}},
                   os.path.join(outdir, f"final{rank}.pt"))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


@pytest.mark.parametrize("world", [2, 1])  # W = 1: the in-line applies
def test_async_xgmi_midrun_checkpoint_is_consistent(tmp_path, world):
    """a mid-run async checkpoint must carry the PS step counters the native service
    advanced (beta powers consistent with the manifest's t) and a snapshot taken with the
    service paused; the final one equals the services' end state."""
    import json
    import torch.multiprocessing as mp
    from safetensors.torch import load_file
    # the step-3 save runs while the peer's pushes are being served (it must neither deadlock
    # against the peer nor tear the PS state); the end-of-run save overwrites it and is checked
    mp.spawn(_ckpt_rank, args=(world, free_port(), str(tmp_path), dict(checkpoint_every=3)),
             nprocs=world, join=True)
    man = json.load(open(tmp_path / "ck" / "manifest.json"))
    final = {}
    for r in range(world):
        final.update(torch.load(tmp_path / f"final{r}.pt")["t"])
    assert {int(k): v for k, v in man["ps_t"].items()} == final   # the end-of-run save
    assert all(t == world * 6 for t in final.values())
    for p in range(man["num_ps"]):
        d = load_file(str(tmp_path / "ck" / f"ps{p}.safetensors"))
        b1 = float(d["ParameterServer/beta1_power"][0])
        assert b1 == pytest.approx(0.9 ** man["ps_t"][str(p)], rel=1e-5)
        for k, v in d.items():
            assert torch.isfinite(v).all(), k


@pytest.mark.parametrize("fault", ["kill@1:3", "stop@1:3"])
def test_xgmi_job_survivor_exits_when_a_peer_fails(tmp_path, fault):
    """SURVEY.md §5.3 on the GPU data plane: two processes on one card over the xGMI exchange;
    rank 1 dies (os._exit) or hangs (SIGSTOP) at step 3.  Rank 0's bucket kernels stop waiting
    after DDL_XGMI_TIMEOUT_S (4 s in tests/fault_rank.py: the kernel records an error word and
    runs to completion, no GPU hang), the runner raises at its next step, and the process ends
    non-zero — within the timeout + the step watchdog (12 s) + abort grace, never a hang."""
    from test_fault_injection_cpu import launch, logs, wait_survivors
    procs = launch(tmp_path, 2, "xgmi", fault)
    codes = wait_survivors(procs, 1, 4.0 + 12.0 + 5.0 + 90.0)  # + import torch / HIP init
    assert 0 in codes, ("rank 0 still running", logs(tmp_path, 2))
    assert codes[0][0] != 0, logs(tmp_path, 2)


def _eval_rank(rank, world, port, outdir):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DDL_DIST_BACKEND="gloo",
                      DDL_XGMI_TIMEOUT_S="20")
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed()
        cfg = TrainConfig(mode="sync", shard="flat", steps=30, batch_size=100, eval_every=10,
                          engine="hip", quiet=True, data_sharding="stride",
                          exchange_backend="xgmi", eval_async=True, watchdog_s=120.0)
        tr = Trainer(cfg, env, dataset=synthetic_mnist(3000, 500, seed=5))
        s = tr.train()
        torch.save({"acc": s["final_acc"], "evals": len(tr.history)},
                   os.path.join(outdir, f"eval{rank}.pt"))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


def test_xgmi_sync_with_side_stream_eval_completes(tmp_path):
    """W = 2 sync over xGMI with the periodic eval on a side stream (the bench's time-to-
    accuracy configuration at W > 1): the training stream must not be a high-priority stream,
    or the comm stream's READY gate can share its hardware queue and wait behind the very launch
    that releases it (this job stalled before the AsyncEvaluator's training stream went to
    normal priority)."""
    import torch.multiprocessing as mp
    mp.spawn(_eval_rank, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        rec = torch.load(os.path.join(tmp_path, f"eval{r}.pt"))
        assert rec["evals"] >= 3 and rec["acc"] > 0.1
