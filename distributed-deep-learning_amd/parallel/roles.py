"""Training roles: ``Single``, ``SyncWorker``/``AsyncWorker`` with co-located ``ParameterServer``s.

Reference roles: ``Single(epoch, batch).train()`` (``*/single.py:3-21``),
``SyncWorker(batch[, rank, num_ps, num_workers]).work(cnt)`` (``*/worker.py``) and
``ParameterServer(params[, rank, num_ps, num_workers]).update()``
(``*/parameter_server.py``), launched MPMD as P PS ranks + W worker ranks.

MI355X layout: one process per GPU.  Every process is a worker; PS ``p`` is hosted by
process ``p % W`` (RCCL cannot place two ranks of one communicator on one GPU).  The
``Trainer`` below wires an engine (HIP kernels, or the torch oracle on CPU), a shard
plan, the hosted ``ParameterServer`` objects and a sync or async exchange, and runs the
reference's loop: 1 epoch x 500 steps of batch 100, test-set accuracy every 10 steps,
final accuracy and ``Time``.
"""
from __future__ import annotations

import contextlib
import sys
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..config import TrainConfig
from ..models import make_engine, engine_segments
from ..models.mnist_cnn import init_params_
from ..ops import rng
from ..ops.adam import AdamHyper
from ..utils import metrics
from ..utils.data import Dataset, get_dataset, batch_indices
from ..utils.watchdog import Watchdog
from ..utils import checkpoint as ckpt
from ..utils.tracing import trace_range
from .comm import DistEnv, SyncExchange, AsyncExchange, init_distributed
from .native_exchange import make_sync_exchange
from .ps import ParameterServer
from .sharding import async_groups, make_plan, segment_aligned_num_ps


def _job_id(env: DistEnv) -> str:
    """Name prefix of this job's POSIX shm segments (mailboxes, completion counters): unique
    per job on the host.  Rank 0 draws a nonce and broadcasts it, so two jobs with the same
    MASTER_PORT (or none, at W = 1) never share (or unlink) each other's segments."""
    import os
    import secrets
    nonce = [f"{os.getpid():x}{secrets.token_hex(4)}"]
    if env.world > 1:
        dist.broadcast_object_list(nonce, src=0)
    return f"ddl{nonce[0]}"


def resolve_num_ps(cfg: TrainConfig, world: int) -> int:
    if cfg.mode == "single" or cfg.shard == "none":
        return 1
    return cfg.num_ps or world


class Trainer:
    """One process = one GPU = one worker (+ the PS shards it hosts)."""

    ABORT_GRACE_S = 5.0  # watchdog: longest wait for ncclCommAbort before os._exit

    def __init__(self, cfg: TrainConfig, env: Optional[DistEnv] = None,
                 dataset: Optional[Dataset] = None):
        self.cfg = cfg
        self.env = env or init_distributed()
        env = self.env
        W, r = env.world, env.rank
        if cfg.mode == "single" and W != 1:
            raise ValueError("mode 'single' runs in one process")
        self.num_ps = resolve_num_ps(cfg, W)
        segs = engine_segments(cfg.engine, env.device)
        asyncm = cfg.mode == "async"
        # One worker and its own PS (async, W = 1): every push is applied before the worker's
        # next step, so the PS parameters ARE the worker's and the math is the sync PS's (one
        # Adam step per push, test_async_single_worker_equals_sync).  Run it on the sync step
        # path — the native runner with the update as the optimizer tail of the backward —
        # instead of a private PS copy plus a copy back per step (0.366 vs 0.307 ms/step), and
        # with the sync path's per-segment buckets (one end-of-step update instead of the
        # backward's optimizer tails: 0.307 vs 0.300).  Not with --ref-quirks (Q4: the PS
        # starts from its own init) or an explicit exchange backend (--exchange xgmi / rccl:
        # the W = 1 rehearsals of the async data planes).
        self.async_as_sync = (asyncm and W == 1 and not cfg.ref_quirks
                              and cfg.exchange_backend == "auto")
        sync_step = cfg.mode == "sync" or self.async_as_sync
        buckets = segs if (cfg.shard == "flat" and cfg.overlap and sync_step) else None
        shard = "none" if cfg.mode == "single" else cfg.shard
        # Async flat plan: every PS range inside one backward segment, so each shard is pushed
        # right after its segment and only the last segment's (52 K-element) shards remain on
        # the step's critical path; needs a PS per segment (P a multiple of W with balanced
        # hosts unless --num-ps sets it, sharding.segment_aligned_num_ps).
        aligned = (asyncm and not self.async_as_sync and cfg.shard == "flat" and cfg.overlap
                   and len(segs) > 1)
        if aligned:
            groups = async_groups(segs)
            self.num_ps = cfg.num_ps or segment_aligned_num_ps(W, groups)
            aligned = self.num_ps >= len(groups)
            if not cfg.num_ps and env.rank == 0 and not cfg.quiet:
                print(f"[ddl_amd] async flat plan: {self.num_ps} segment-aligned PS "
                      f"(--num-ps not given)", file=sys.stderr)
            buckets = groups if aligned else None
        self.plan = make_plan(shard, self.num_ps, buckets=buckets, segment_aligned=aligned)
        dev = env.device
        self.params = torch.zeros(self.plan.total, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(self.plan.total, dtype=torch.float32, device=dev)
        # Same seed on every rank -> identical initial parameters (the reference
        # initialises every process independently; --ref-quirks).
        init_seed = cfg.seed + (r if cfg.ref_quirks else 0)
        init_params_(self.params, self.plan.tensor_offsets, init_seed)
        self.engine = make_engine(cfg.engine, self.params, self.grads, self.plan.tensor_offsets,
                                  dev, cfg.batch_size, graph=cfg.graph)
        hyper = AdamHyper(lr=cfg.lr)
        hosted = [p for p in range(self.num_ps) if self.plan.host_rank(p, W) == r]
        self.servers: Dict[int, ParameterServer] = {}
        for p in hosted:
            own = None
            if asyncm and not self.async_as_sync:
                own = self.params
                if cfg.ref_quirks:  # PS initialised independently of the workers (Q4)
                    tmp = torch.zeros_like(self.params)
                    init_params_(tmp, self.plan.tensor_offsets, cfg.seed + 10007 + p)
                    own = tmp
            self.servers[p] = ParameterServer(self.plan, p, dev, hyper, cfg.optimizer,
                                              cfg.momentum, own_params=own,
                                              native_optim=self.engine.name != "torch")
        self.data = dataset if dataset is not None else get_dataset(cfg.data, seed=1234)
        self.data = self.data.to(dev)
        self.steps = cfg.steps or (self.data.total_batch // cfg.batch_size)
        if asyncm and not self.async_as_sync:
            self.exchange = self._make_async_exchange(cfg, env)
            if hasattr(self.exchange, "attach_runner"):
                self.exchange.attach_runner(self.engine, segs)
        else:
            self.exchange = make_sync_exchange(self.plan, env, self.params, self.grads, segs,
                                               self.servers, self.engine, cfg, hyper)
        self.log = metrics.JsonlLogger(cfg.log_jsonl, r)
        self.global_step = 0
        self.history: List[dict] = []

    def _make_async_exchange(self, cfg: TrainConfig, env: DistEnv):
        """The async data plane.  On a GPU: the xGMI peer-memory exchange (``async_xgmi.py``,
        no p2p kernels at all) when asked for, or by default at W > 1 with the HIP engine; else
        point-to-point RCCL in exclusive sessions (``async_rccl.py``, deadlock-free under any
        stream-to-hardware-queue mapping).  The round-2 Python RCCL pair-group exchange, whose
        concurrent p2p kernels could block each other's hardware queues, is NOT a GPU fallback
        any more; it remains the CPU (gloo) implementation."""
        steps = self.steps * cfg.epochs
        job = _job_id(env)
        cuda = env.device.type == "cuda"
        want_xgmi = cfg.exchange_backend == "xgmi" or (
            cfg.exchange_backend == "auto" and env.world > 1 and self.engine.name == "hip")
        import sys
        if want_xgmi and cuda:
            from .async_xgmi import AsyncPeerExchange, AsyncPeerUnavailable
            try:
                return AsyncPeerExchange(self.plan, env, self.params, self.grads, self.servers,
                                         steps_per_worker=steps, grad_reduce=cfg.grad_reduce,
                                         check_provenance=cfg.check_provenance,
                                         optimizer=cfg.optimizer, job_id=job)
            except AsyncPeerUnavailable as e:
                if env.rank == 0:
                    print(f"[ddl_amd] async xGMI exchange unavailable ({e}); using RCCL sessions",
                          file=sys.stderr)
        if cuda:
            from .async_rccl import RcclAsyncExchange, RcclAsyncUnavailable
            try:
                return RcclAsyncExchange(self.plan, env, self.params, self.grads, self.servers,
                                         steps_per_worker=steps, job_id=job,
                                         optimizer=cfg.optimizer,
                                         check_provenance=cfg.check_provenance)
            except RcclAsyncUnavailable as e:
                if env.world > 1 and env.backend == "nccl":
                    raise RuntimeError(f"async mode on GPU: neither the xGMI nor the RCCL-"
                                       f"session exchange is available ({e})") from e
                # a non-RCCL default group (the shared-GPU gloo rehearsal after an xGMI set-up
                # failure) keeps the host-driven exchange, as before round 3
                print(f"[ddl_amd] async RCCL-session exchange unavailable ({e}); using the "
                      f"host-driven exchange", file=sys.stderr)
        return AsyncExchange(self.plan, env, self.params, self.grads, self.servers,
                             steps_per_worker=steps, grad_reduce=cfg.grad_reduce,
                             check_provenance=cfg.check_provenance, job_id=job)

    # ---- one worker step (reference SyncWorker.work + pull + assign) -----------------------------
    def batch(self, step: int):
        lo, hi = batch_indices(step, self.cfg.batch_size, self.data.total_batch, self.env.rank,
                               self.env.world, self.cfg.data_sharding)
        return self.data.x_train[lo:hi], self.data.y_train[lo:hi]

    def train_step(self, step: int) -> None:
        cfg = self.cfg
        x, y = self.batch(step)
        seed = rng.step_seed(cfg.seed, self.env.rank, self.global_step)
        if cfg.mode == "async" and not self.async_as_sync and \
                getattr(self.exchange, "runner", None) is not None:
            with trace_range("step_native_async"):
                self.exchange.native_step(self.engine, x, y, cfg.keep_prob, seed)
        elif cfg.mode == "async" and not self.async_as_sync:
            with trace_range("fwd_bwd"):
                self.engine.forward_backward(x, y, cfg.keep_prob, seed)
            with trace_range("push_pull"):
                self.exchange.push_pull()
        elif getattr(self.exchange, "native", False):
            with trace_range("step_native"):
                self.exchange.step(x, y, cfg.keep_prob, seed)
        else:
            ex = self.exchange
            ex.begin_step()
            with trace_range("fwd_bwd"):
                self.engine.forward_backward(x, y, cfg.keep_prob, seed, on_segment=ex.grads_ready)
            with trace_range("exchange"):
                ex.finish_step()
        self.global_step += 1

    def evaluate(self) -> float:
        """Test-set accuracy.  The reference has every worker score the full 10k test set
        (``mnist_sync/worker.py:71-72``); in sync mode the ranks run in lockstep anyway, so
        each scores 1/W of it and one all-reduce of the correct counts gives the identical
        number W times faster (eval dominates time-to-accuracy)."""
        with trace_range("eval"):
            x, y = self.data.x_test, self.data.y_test
            env = self.env
            if not (self.cfg.dist_eval and self.cfg.mode == "sync" and env.world > 1):
                return self.engine.accuracy(x, y)
            n = x.shape[0]
            per = (n + env.world - 1) // env.world
            lo, hi = min(n, env.rank * per), min(n, (env.rank + 1) * per)
            c = self.engine.correct(x[lo:hi], y[lo:hi]) if hi > lo else 0
            t = torch.tensor([float(c)], dtype=torch.float64, device=env.device)
            dist.all_reduce(t)
            return float(t.item()) / n

    def _on_hang(self) -> None:
        """Watchdog fired: abort the native RCCL communicator (pending collectives return
        with an error instead of spinning) and end the process so the launcher tears the
        job down."""
        import os
        import sys
        import threading
        ab = getattr(self.exchange, "abort", None)
        if ab is not None:
            # ncclCommAbort can itself block (proxy threads, kernels stuck on a dead peer):
            # run it on a daemon thread and exit unconditionally after a bounded join
            def _abort():
                try:
                    ab()
                except Exception as e:  # best effort: we are exiting anyway
                    sys.stderr.write(f"[watchdog] comm abort failed: {e}\n")
            t = threading.Thread(target=_abort, name="ddl-comm-abort", daemon=True)
            t.start()
            t.join(timeout=self.ABORT_GRACE_S)
            if t.is_alive():
                sys.stderr.write("[watchdog] comm abort still blocked; exiting anyway\n")
                sys.stderr.flush()
        os._exit(124)

    # ---- reference main loop -----------------------------------------------------------------------
    def train(self) -> dict:
        cfg, env = self.cfg, self.env
        clock = metrics.Clock()
        single = cfg.mode == "single"
        # Resume continues the run (reference loop mnist_sync/worker.py:58-72): the restored
        # global step is the position in the epoch loop, so the data index (cnt), the eval
        # cadence (cnt % eval_every) and the dropout seeds (global_step) all pick up where the
        # checkpointed run stopped — a resumed run is the uninterrupted run, not a new epoch.
        if cfg.resume and cfg.checkpoint_dir:
            ckpt.load(self, cfg.checkpoint_dir)
        first = self.global_step
        last = cfg.epochs * self.steps
        if cfg.max_steps is not None:
            last = min(last, cfg.max_steps)
        asyncx = cfg.mode == "async" and not self.async_as_sync
        if asyncx:
            # the PS services expect exactly this run's pushes (every worker runs the same
            # window), and resume their step counters from the checkpoint (load above)
            self.exchange.steps = max(0, last - first)
            self.exchange.start()
        wd = Watchdog(cfg.watchdog_s, name=f"rank{env.rank}", on_timeout=self._on_hang)
        t_target = None
        train_wall = 0.0

        def on_eval(meta, acc, wall):
            nonlocal t_target
            if not cfg.quiet:
                line = (metrics.single_progress(meta["epoch"], meta["cnt"], acc) if single else
                        metrics.worker_progress(env.rank, meta["epoch"], meta["cnt"], acc))
                metrics.emit(line)
            self.log.log(event="eval", epoch=meta["epoch"], batch=meta["cnt"], acc=acc,
                         wall=wall, step=meta["step"])
            self.history.append({"step": meta["step"], "acc": acc, "wall": wall})
            if cfg.target_acc is not None and t_target is None and acc >= cfg.target_acc:
                t_target = wall

        aeval = None
        if cfg.eval_async and cfg.eval_every and getattr(self.engine, "name", "") == "hip":
            from .async_eval import AsyncEvaluator
            aeval = AsyncEvaluator(self, on_result=on_eval)
            torch.cuda.synchronize()
            clock = metrics.Clock()
        # with the side-stream eval, training runs on the evaluator's training stream (NORMAL
        # priority: the native runners' gates need it off the high-priority queue pool)
        train_ctx = (torch.cuda.stream(aeval.train_stream) if aeval is not None
                     else contextlib.nullcontext())
        with train_ctx:
            if aeval is not None:
                aeval.start()
            for epoch in range(cfg.epochs):
                if (epoch + 1) * self.steps <= first:
                    continue
                if self.global_step >= last:
                    break
                for cnt in range(self.steps):
                    if epoch * self.steps + cnt < first:
                        continue  # done before the checkpoint
                    if self.global_step >= last:
                        break
                    t0 = time.perf_counter()
                    self.train_step(cnt)
                    wd.kick()
                    if aeval is not None:
                        if cnt % cfg.eval_every == 0:
                            aeval.submit({"epoch": epoch, "cnt": cnt, "step": self.global_step})
                        aeval.poll()
                        train_wall += time.perf_counter() - t0
                    elif cfg.eval_every and cnt % cfg.eval_every == 0:
                        if env.device.type == "cuda":
                            torch.cuda.synchronize()
                        train_wall += time.perf_counter() - t0
                        acc = self.evaluate()
                        on_eval({"epoch": epoch, "cnt": cnt, "step": self.global_step}, acc,
                                clock.wall())
                    else:
                        train_wall += time.perf_counter() - t0
                    if cfg.checkpoint_dir and cfg.checkpoint_every and \
                            self.global_step % cfg.checkpoint_every == 0:
                        ckpt.save(self, cfg.checkpoint_dir)
        if aeval is not None:
            torch.cuda.current_stream().wait_stream(aeval.train_stream)
            aeval.drain()
            aeval.close()  # its streams and its eval engine's workspace, now
        if asyncx:
            self.exchange.join()
            if cfg.check_provenance:
                self.exchange.verify_provenance()
        # drain first: the last steps' exchange kernels may still be running, and a bounded
        # xGMI wait that times out records its error only when it gives up
        if env.device.type == "cuda":
            torch.cuda.synchronize()
        if getattr(self.exchange, "native", False) and env.world > 1:
            self.exchange.check()
        if env.world > 1:
            dist.barrier()
        cpu_t, wall_t = clock.cpu(), clock.wall()
        acc = self.evaluate()
        if not cfg.quiet:
            metrics.emit(metrics.single_final(acc) if single else metrics.worker_final(env.rank, acc))
            metrics.emit(metrics.time_line(cpu_t))
        wd.stop()
        if cfg.checkpoint_dir:
            ckpt.save(self, cfg.checkpoint_dir)
        imgs = (self.global_step - first) * cfg.batch_size  # this run's steps (resume)
        summary = dict(final_acc=acc, cpu_time=cpu_t, wall_time=wall_t, train_wall=train_wall,
                       images=imgs, images_per_s=imgs / max(train_wall, 1e-9),
                       time_to_target=t_target, steps=self.global_step, plan=self.plan.describe())
        self.log.log(event="final", **summary)
        if asyncx:
            self.exchange.close()
        return summary


def close_trainers(trainers, env: DistEnv) -> None:
    """Tear down the native communicators of these trainers on every rank in the same order,
    between barriers (a finalisation that synchronises with the peers must not wait on a rank
    still computing, and garbage collection would destroy them at rank-dependent moments)."""
    if env.world > 1:
        if env.device.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier()
    for t in trainers:
        # native sync runners and the asynchronous data planes (xGMI / RCCL); the Python sync
        # exchange has nothing native to release
        close = getattr(t.exchange, "close", None)
        if close is not None and (getattr(t.exchange, "native", False)
                                  or t.cfg.mode == "async"):
            close()
    if env.world > 1:
        dist.barrier()


class Single(Trainer):
    """``Single(epoch, batch_size).train()`` — reference ``mnist_sync/single.py:3-21``."""

    def __init__(self, epoch: int = 1, batch_size: int = 100, **kw):
        cfg = TrainConfig(mode="single", shard="none", epochs=epoch, batch_size=batch_size, **kw)
        super().__init__(cfg, DistEnv(device=torch.device("cuda") if torch.cuda.is_available()
                                      else torch.device("cpu")))
