#!/usr/bin/env python3
"""Headline benchmark: MNIST CNN, synchronous sharded parameter server, images/s (whole job).

Config (BASELINE.json): ``mnist_sync_sharding`` — W workers (one per MI355X), one PS shard
per GPU co-located with the workers, the parameters and Adam state sharded into contiguous
byte-equal chunks of each gradient bucket so that push/pull are one RCCL reduce-scatter +
all-gather per bucket (``--shard flat``; in sync mode every policy computes the same update,
the policy only changes who applies it and the traffic pattern — the reference's
tensor-granular ``contiguous``/``greedy`` planners are ``--shard contiguous|greedy``),
batch 100 per worker (``mnist_sync/worker.py:42``),
Adam 1e-4 on the PS (``model.py:93``), dropout keep 0.5, fp32 (the reference computes in
fp32 throughout; gfx950 fp32 MFMA), synthetic MNIST-shaped data resident in HBM and
random (TF1 glorot) init.  Weak scaling: per-GPU batch fixed at 100, so the global batch
is 100*W.  A timed step is the full worker step: batch fetch, forward, backward,
gradient push (RCCL), PS Adam update, parameter pull — eval excluded.

Usage:  python bench.py [--gpus N --steps K --warmup W]
  N>1:  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
            --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# device-memory kernel arguments and dmabuf IPC before any HIP initialisation (see
# ddl_amd/__init__)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

METRIC = "images/sec (whole node) + time-to-target-acc, MNIST CNN sync-sharding at 1/2/4/8 MI355X"
# Baseline per GPU (the reference publishes no numbers): the strongest stock
# PyTorch-ROCm version of the same step measured on MI355X — MIOpen-autotuned convs, fused
# Adam, the whole step captured as one HIP graph (scripts/torch_best_baseline.py, round 2:
# 0.8464 ms/step).  The round-1 faithful-semantics eager baseline (bench.py --engine torch,
# 51,308.5 img/s) is 2.3x slower still.
BASELINE_IMG_PER_S_PER_GPU = 118145.4


def variant_of(mode: str, policy: str) -> str:
    """The reference directory whose semantics the run has; the flat and
    LPT plans are this framework's sharding policies for the sharded variants."""
    base = {"none": "mnist_{}", "contiguous": "mnist_{}_sharding",
            "greedy": "mnist_{}_sharding_greedy"}.get(policy)
    if base:
        return base.format(mode)
    return f"mnist_{mode}_sharding ({policy} plan)"


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch-size", type=int, default=100)
    ap.add_argument("--shard", default="flat",
                    choices=["none", "contiguous", "greedy", "lpt", "flat"],
                    help="PS shard policy (default flat: one PS per GPU owning a byte-equal "
                         "contiguous chunk of every gradient bucket -> RCCL reduce-scatter + "
                         "all-gather, BASELINE.json config; 'contiguous'/'greedy' are the "
                         "reference's tensor-granular planners -> grouped reduce + broadcast)")
    ap.add_argument("--mode", default="sync", choices=["sync", "async"])
    ap.add_argument("--engine", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--graph", action="store_true",
                    help="replay the engine step as HIP graphs (measured slower than eager "
                         "stream launches on MI355X: 0.600 vs 0.552 ms/step)")
    ap.add_argument("--no-graph", action="store_true", help="(default; kept for compatibility)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-native-exchange", action="store_true",
                    help="Python-driven exchange instead of the C++ SyncRunner")
    ap.add_argument("--force-collectives", action="store_true",
                    help="W = 1 rehearsal of the multi-GPU step: keep the reduce-scatter / "
                         "all-gather units on a 1-rank RCCL communicator (comm stream, events, "
                         "RCCL launches) instead of the local update; with --exchange xgmi the "
                         "fused xGMI bucket kernels (every push to itself) instead")
    ap.add_argument("--exchange", default="auto", choices=["auto", "rccl", "xgmi"],
                    help="W > 1 data plane of the native sync runner: RCCL reduce-scatter / "
                         "all-gather, or the fused xGMI peer-memory exchange (one push / "
                         "owner-Adam / pull kernel per bucket).  auto: both are set up and "
                         "timed on a short A/B before the warmup, the faster one is benchmarked "
                         "(both timings are reported)")
    ap.add_argument("--ab-steps", type=int, default=30,
                    help="timed steps per candidate of the --exchange auto A/B")
    ap.add_argument("--splits", default=None, help="comma-separated split-K factors per op")
    ap.add_argument("--tta", type=float, default=0.95,
                    help="after the throughput run, train one reference epoch (500 steps/worker, "
                         "full test-set eval every 10 steps, eval time included) and report the "
                         "wall time to this test accuracy; <= 0 skips it")
    ap.add_argument("--tta-steps", type=int, default=None,
                    help="steps per worker of the time-to-accuracy run (default: one reference "
                         "epoch, 500)")
    ap.add_argument("--no-tta-hard", action="store_true",
                    help="skip the time-to-accuracy run on the hard synthetic set "
                         "(utils/data.py synthetic_mnist_hard; default: run it too)")
    ap.add_argument("--tta-sync-eval", action="store_true",
                    help="time-to-accuracy run with the eval in line on the training stream "
                         "(default on GPU: side-stream eval from parameter snapshots)")
    ap.add_argument("--prewarm-steps", type=int, default=-1,
                    help="untimed training steps BEFORE the --warmup steps (reported in the "
                         "JSON; default 1000 on a GPU, 0 on CPU).  Measured on MI355X: after 5 warmup steps a 20-step window "
                         "runs 0.321-0.323 ms/step, after 100 0.308-0.312 (the GPU is still "
                         "ramping up); round 5, the driver's --steps 20 --warmup 5 on one box, 4 "
                         "alternating rounds: prewarm 100 0.2967-0.2979, 300 0.2958-0.3012, 1000 "
                         "0.2955-0.2965 ms/step (profiles/r5_driver_window_prewarm.txt)")
    ap.add_argument("--extra-plans", default="contiguous",
                    help="W > 1 sync: comma-separated shard plans also timed after the headline "
                         "plan (same steps), reported under 'plans' (BASELINE config 3 names "
                         "contiguous shards); empty string skips them")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import init_distributed
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import synthetic_mnist

    env = init_distributed()
    world = env.world
    if a.gpus != world and not (a.gpus == 1 and world == 1):
        if env.rank == 0:
            print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    cuda = env.device.type == "cuda"
    n_pre = a.prewarm_steps if a.prewarm_steps >= 0 else (1000 if cuda else 0)
    total_steps = n_pre + a.warmup + a.steps
    data = synthetic_mnist()

    def make_trainer(backend, shard=None, native=None):
        cfg = TrainConfig(mode=a.mode, shard=shard or a.shard, steps=total_steps,
                          batch_size=a.batch_size,
                          eval_every=0, engine=a.engine, graph=a.graph and not a.no_graph,
                          overlap=not a.no_overlap, quiet=True, data_sharding="stride",
                          native_exchange=(not a.no_native_exchange) if native is None else native,
                          force_collectives=a.force_collectives, exchange_backend=backend)
        t = Trainer(cfg, env, dataset=data)
        if a.splits and hasattr(t.engine, "set_splits"):
            t.engine.set_splits([int(s) for s in a.splits.split(",")])
        return t

    def sync():
        if cuda:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def backend_of(t) -> str:
        ex = t.exchange
        if getattr(t, "async_as_sync", False):
            return "native-local (async W=1 as sync)"
        if a.mode == "async":
            if getattr(ex, "backend", "") != "xgmi":
                return type(ex).__name__
            svc = getattr(ex, "service_mode", None)  # PS side: the native host service
            return ("native-" if getattr(ex, "runner", None) is not None else "python-") + \
                "xgmi-async" + (" (in-line applies)" if svc == "inline" else
                                f" ({svc} service)" if svc else "")
        if not getattr(ex, "native", False):
            return "python"
        return "native-" + getattr(ex, "backend", "rccl")

    # W > 1, sync, flat plan: the xGMI exchange is a candidate next to RCCL.  With several ranks
    # on one GPU (DDL_DIST_BACKEND=gloo rehearsal) RCCL cannot run, so xgmi is the only one.
    shared_gpu = os.environ.get("DDL_DIST_BACKEND", "") == "gloo" and cuda
    candidates = [a.exchange]
    if a.exchange == "auto" and world > 1 and a.mode == "sync" and a.shard == "flat" and cuda:
        candidates = ["xgmi"] if shared_gpu else ["rccl", "xgmi"]
    if os.environ.get("DDL_AB_CANDIDATES") and world > 1:  # test hook: force an A/B list
        candidates = os.environ["DDL_AB_CANDIDATES"].split(",")
    ab = {}
    tr = None
    # every trainer built here stays referenced until the process ends: a garbage-collected
    # runner would destroy its RCCL communicator / IPC mappings at a different moment on each
    # rank
    keep = []
    def digest(p):
        """Bit-exact digest of a parameter replica: sum of the raw fp32 bit patterns (int64,
        exact) and whether every value is finite."""
        bits = int(p.view(torch.int32).to(torch.int64).sum().item())
        return bits, bool(torch.isfinite(p).all().item())

    def replicas_consistent(t) -> bool:
        """Sync PS: every worker pulled the same parameters, so the replicas must be bitwise
        equal on all ranks and finite (collective)."""
        dg = [digest(t.params)]
        if world > 1:
            dg = [None] * world
            dist.all_gather_object(dg, digest(t.params))
        return all(d[1] for d in dg) and len({d[0] for d in dg}) == 1

    if len(candidates) > 1:
        # short A/B before the benchmark proper (a wait that times out in the xGMI path raises
        # at the next step on that rank; every rank votes, so a failed candidate is dropped
        # by all ranks together).  Each candidate is also checked for correctness: in a sync
        # PS step every worker pulls the same parameters, so the replicas must be bitwise equal
        # on all ranks, finite, and (same init, data and step count) close to the first
        # candidate's — a data plane that loses or tears an update fails here, not silently.
        best, ref_params = None, None
        for c in candidates:
            try:
                t = make_trainer(c)
                keep.append(t)
            except Exception as e:  # noqa: BLE001 - reported, not fatal for the other candidate
                ab[c] = {"error": str(e)[:200]}
                t = None
            ok, ms = t is not None, None
            if ok:
                try:
                    p0 = t.params.clone()
                    # untimed steps first: the first candidate would otherwise run on a cold GPU
                    # (clocks ramp over ~100 steps); the same count for every candidate, so their
                    # replicas stay comparable (same init, data and step count)
                    nw = 5 + min(200, n_pre)
                    for i in range(nw):
                        t.train_step(i)
                    sync()
                    t0 = time.perf_counter()
                    for i in range(nw, nw + a.ab_steps):
                        t.train_step(i)
                    sync()
                    ms = 1e3 * (time.perf_counter() - t0) / a.ab_steps
                    if hasattr(t.exchange, "check"):
                        t.exchange.check()
                except RuntimeError as e:
                    ok = False
                    ab[c] = {"error": str(e)[:200]}
            votes = [None] * world
            dist.all_gather_object(votes, bool(ok))
            if not all(votes):
                ab.setdefault(c, {"error": "failed on some rank"})
                continue
            ms = max_over_ranks(ms)
            ab[c] = {"ms_per_step": round(ms, 4), "exchange": backend_of(t)}
            good = replicas_consistent(t)
            rel = None
            if ref_params is None:
                ref_params = (t.params.clone(), p0)
            else:
                moved = (ref_params[0] - ref_params[1]).abs().mean()
                rel = float(((t.params - ref_params[0]).abs().mean() / moved.clamp_min(1e-30)).item())
                rel = max_over_ranks(rel)
                good = good and rel < 0.1
                ab[c]["mean_diff_vs_" + candidates[0]] = round(rel, 5)
            ab[c]["replicas_consistent"] = good
            if not good:
                continue
            if best is None or ms < best[0]:
                best = (ms, c, t)
        if best is not None:
            chosen = best[1]
        else:
            ran = [c for c in candidates if "ms_per_step" in ab.get(c, {})]
            if not ran:
                raise RuntimeError(f"no exchange candidate worked: {ab}")
            chosen = ran[0]
            ab["note"] = "no candidate passed the replica check; benchmarking the first that ran"
        # a fresh trainer for the benchmark proper: identical initial state for every choice
        tr = make_trainer(chosen)
    else:
        chosen = candidates[0]
        tr = make_trainer(chosen)
    keep.append(tr)
    cfg = tr.cfg
    # W > 1 (or the forced 1-rank rehearsal), sync, native runner: prove the READY-flag hand-off
    # on this job before the timed run (bit-identical to the event hand-off on every rank, else
    # every rank falls back to the events); the verdict goes into the JSON config
    handoff = None
    if (a.mode == "sync" and hasattr(tr.exchange, "handoff_check")
            and (world > 1 or a.force_collectives)):
        from ddl_amd.parallel.native_exchange import NativeUnavailable
        try:
            handoff = tr.exchange.handoff_check(tr)
        except NativeUnavailable as e:
            # the replicas diverged under the reference (event) hand-off on this data plane: it
            # is refused on every rank (handoff_vote raises everywhere) and the job continues on
            # the Python exchange (torch.distributed collectives)
            from ddl_amd.parallel.roles import close_trainers
            close_trainers([tr], env)
            keep.remove(tr)
            handoff = {"handoff": f"data plane '{chosen}' refused: {str(e)[:160]}"}
            tr = make_trainer(chosen, native=False)
            keep.append(tr)
            cfg = tr.cfg
    replica_check = None

    def timed_run(t):
        """prewarm + warmup (untimed), then exactly a.steps steps between barrier+sync pairs;
        returns the max-over-ranks seconds of the timed window."""
        asyncx = a.mode == "async" and not getattr(t, "async_as_sync", False)
        if asyncx:
            t.exchange.steps = total_steps
            t.exchange.start()
        for i in range(n_pre + a.warmup):
            t.train_step(i)
        sync()
        if a.mode == "sync" and world > 1 and t is tr:
            # the replicas of a synchronous PS step must be bitwise equal on every rank: checked
            # for the benchmarked data plane whether it was chosen by the A/B or named explicitly
            nonlocal replica_check
            replica_check = replicas_consistent(t)
            if not replica_check:
                raise RuntimeError(f"sync replicas diverge across ranks on the "
                                   f"'{backend_of(t)}' data plane: refusing to benchmark it")
            sync()
        t0 = time.perf_counter()
        for i in range(n_pre + a.warmup, total_steps):
            t.train_step(i)
        if asyncx:
            t.exchange.join()
        sync()
        return max_over_ranks(time.perf_counter() - t0)

    elapsed = timed_run(tr)
    ms = 1e3 * elapsed / a.steps
    imgs = world * a.batch_size * a.steps / elapsed
    acc = tr.evaluate()

    # W > 1 sync: the reference's tensor-granular plans on the same harness (RCCL grouped
    # reduce / broadcast; contiguous puts 59 % of the bytes on the last PS at W = 8)
    plans = {}
    extra = [p for p in a.extra_plans.split(",") if p and p != a.shard]
    if world > 1 and a.mode == "sync" and extra:
        # each plan over RCCL (grouped reduce / broadcast) and over the xGMI owner buckets (one
        # push / owner update / pull kernel per unit); a shared-GPU rehearsal has no RCCL
        for p in extra:
            for be in (["xgmi"] if shared_gpu else ["rccl", "xgmi"]):
                key = p if be == "rccl" or shared_gpu else f"{p}/xgmi"
                try:
                    t = make_trainer(be, shard=p)
                    keep.append(t)
                    el = timed_run(t)
                    plans[key] = {"ms_per_step": round(1e3 * el / a.steps, 4),
                                  "value": round(world * a.batch_size * a.steps / el, 1),
                                  "exchange": backend_of(t), "num_ps": t.num_ps}
                except RuntimeError as e:
                    plans[key] = {"error": str(e)[:200]}

    # the record's facts about the benchmarked trainer, taken before any release below
    engine_name = getattr(tr.engine, "name", a.engine)
    num_ps, policy, exchange_name = tr.num_ps, tr.plan.policy, backend_of(tr)
    # W > 1 (sync, and async after its exchange joined): close and drop every trainer built so
    # far (collectively, between barriers, nothing in flight) before each time-to-accuracy run —
    # close() releases each runner's comm stream, events, flags and peer mappings, the side-
    # stream evaluator its own streams.  Kept alive, they add hardware queues per process; with
    # several processes on ONE card that stalled the time-to-accuracy runs (docs/DESIGN.md,
    # "W = 4 on one card").  DDL_BENCH_RELEASE=0 keeps them to the end as before.
    release = world > 1 and os.environ.get("DDL_BENCH_RELEASE", "1") == "1"

    def release_all():
        import gc
        from ddl_amd.parallel.roles import close_trainers
        close_trainers(keep, env)
        keep.clear()
        gc.collect()
        sync()

    if release:
        t = best = tr = None  # noqa: F841 - drop the last references before the collect
        release_all()

    hard_data = [None]

    def time_to_acc(sharding, hard=False):
        cfg2 = TrainConfig(mode=a.mode, shard=a.shard, batch_size=a.batch_size, eval_every=10,
                           steps=a.tta_steps,
                           engine=a.engine, graph=a.graph and not a.no_graph,
                           overlap=not a.no_overlap, quiet=True, target_acc=a.tta,
                           data_sharding=sharding, native_exchange=not a.no_native_exchange,
                           eval_async=cuda and not a.tta_sync_eval, exchange_backend=chosen)
        if hard and hard_data[0] is None:
            from ddl_amd.utils.data import synthetic_mnist_hard
            hard_data[0] = synthetic_mnist_hard()
        tr2 = Trainer(cfg2, env, dataset=hard_data[0] if hard else data)
        keep.append(tr2)
        s = tr2.train()
        hit = next((h for h in tr2.history if h["acc"] >= a.tta), None)
        if release:
            tr2 = None  # noqa: F841 - the frame's own reference, before the collect
            release_all()
        return {"target_acc": a.tta, "time_to_target_s": s["time_to_target"],
                # the global step of the first eval at the target: convergence without the clock
                # (ranks sharing one card slow the clock, not the steps)
                "steps_to_target": hit["step"] if hit else None,
                "final_acc": round(s["final_acc"], 4), "epoch_wall_s": round(s["wall_time"], 4),
                "steps_per_worker": s["steps"], "eval_every": 10, "data_sharding": sharding,
                "data": "synthetic-hard (utils/data.py HARD)" if hard else "synthetic",
                "eval": ("distributed over ranks" if world > 1 and a.mode == "sync" else "full")
                + ("; side stream from parameter snapshots" if cfg2.eval_async else "; in line")}

    # time to accuracy under the bench's per-worker data shards (stride: worker r takes every
    # W-th batch) and, at W > 1, under the reference protocol (replicate: every worker trains on
    # the same batches, mnist_sync/worker.py:27-28) — identical at W = 1
    # ... and on the hard synthetic set (the default set ends its epoch at
    # 0.998, too easy to show what staleness or the replicate protocol cost in convergence)
    tta, tta_rep, tta_hard, tta_hard_rep = None, None, None, None
    if a.tta is not None and a.tta > 0:
        tta = time_to_acc("stride")
        if world > 1:
            tta_rep = time_to_acc("replicate")
        if not a.no_tta_hard:
            tta_hard = time_to_acc("stride", hard=True)
            if world > 1:
                tta_hard_rep = time_to_acc("replicate", hard=True)

    if env.rank == 0:
        base = BASELINE_IMG_PER_S_PER_GPU
        rec = {
            "metric": METRIC,
            "value": round(imgs, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(imgs / (base * world), 3) if base else None,
            "dtype": "fp32",
            "data": "synthetic (MNIST-shaped, HBM-resident), random glorot init",
            "config": {
                "model": "mnist_cnn 4conv+3fc (2,656,010 params)",
                "global_batch": world * a.batch_size,
                "seq_len": None,
                "parallelism": f"dp{world}-ps{num_ps}-{a.mode}-{policy}",
                "variant": variant_of(a.mode, policy),
                "plan": policy,
                "engine": engine_name,
                "hip_graph": bool(a.graph and not a.no_graph),
                "overlap": not a.no_overlap,
                "exchange": exchange_name,
                "forced_1rank_collectives": bool(a.force_collectives),
                "optimizer": "adam(1e-4) on PS shards",
                # the throughput window's batches: worker r reads batch r, r + W, ... (per-step
                # work and traffic are the same under the reference's replicate protocol)
                "data_sharding": "stride",
                "handoff": (handoff["handoff"] if handoff
                            else "n/a (W = 1, local updates)" if world == 1
                            else "n/a (no native runner)"),
            },
            "test_acc_after_run": round(acc, 4),
            "prewarm": {"steps": n_pre, "note": "untimed steps before the warmup steps: the "
                        "GPU is still ramping up after a few steps (20-step window after 5 "
                        "warmup steps: 0.322 vs 0.308 ms/step after 100; after 1000 the "
                        "20-step window spreads 1 us instead of 1-5 us)"},
        }
        if handoff:
            rec["handoff_check"] = handoff
        if replica_check is not None:
            rec["replicas_bit_identical_before_timing"] = replica_check
        if ab:
            rec["exchange_ab"] = ab
        if plans:
            rec["plans"] = plans
        if shared_gpu and world > 1:
            rec["note"] = (f"{world} ranks share ONE GPU (DDL_DIST_BACKEND=gloo rehearsal): "
                           "functional check of the W > 1 path, not a multi-GPU measurement; "
                           f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'default')} "
                           "per process")
        if tta is not None:
            rec["time_to_acc"] = tta
        if tta_rep is not None:
            rec["time_to_acc_replicate"] = tta_rep
        if tta_hard is not None:
            rec["time_to_acc_hard"] = tta_hard
        if tta_hard_rep is not None:
            rec["time_to_acc_hard_replicate"] = tta_hard_rep
        print(json.dumps(rec), flush=True)
    if world > 1:
        from ddl_amd.parallel.roles import close_trainers
        close_trainers(keep, env)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
