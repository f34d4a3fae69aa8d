"""Asynchronous parameter server over xGMI peer memory (``csrc/kernels/xgmi_async.hip``).

Reference (``mnist_async_sharding/worker.py:30-37,88-94``,
``parameter_server.py:94-111``): each worker Sends its gradient tensors to their PS and
blocks in Recv for the parameters; each PS serves whichever push arrives (``ANY_SOURCE``),
applies Adam with its own step counter and Sends the parameters back to that worker.

MI355X design (no host staging, no RCCL pair communicators):

* worker step: push kernels store each PS shard of the gradient into the PS host's inbox
  slot for this worker (remote stores over xGMI) and post every slice on the ARRIVAL BOARD in
  host memory shared by all ranks; the worker then waits — like the reference's blocking
  Recv — until every PS has stored the new parameters back (completion counters in the same
  shared segment);
* PS host: a native service thread scans the board and enqueues, on its PS stream, one
  ``apply`` kernel per completed push in the order it sees them (the ``ANY_SOURCE`` order):
  Adam on the PS's private copy (one step of its counter per arrival, atomic per shard —
  fixing the reference's per-tag mixing race Q3), store the shard into the worker's parameter
  buffer, bump the worker's completion counter.  The host never touches the data.

No kernel waits for another kernel (the kernel file says why that matters: HIP multiplexes
streams onto a few hardware queues), so no interleaving of workers and PS streams can
deadlock.  Staleness is one round per worker, as in the reference.

Works with several processes on ONE GPU (IPC does, RCCL does not), so the async W > 1 path is
tested on a one-GPU box (``tests/test_xgmi_gpu.py``).
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import native
from .comm import DistEnv
from .ps import ParameterServer
from .sharding import ShardPlan


class AsyncPeerUnavailable(RuntimeError):
    pass


class _RunnerCounters:
    """The runner's in-line step counters behind the service's ``t(ps)``."""

    def __init__(self, runner):
        self.t = runner.inline_t


class AsyncPeerExchange:
    backend = "xgmi"

    def __init__(self, plan: ShardPlan, env: DistEnv, params: torch.Tensor, grads: torch.Tensor,
                 servers: Dict[int, ParameterServer], steps_per_worker: int,
                 grad_reduce: str = "sum", job_id: str = "ddl",
                 check_provenance: bool = False, optimizer: str = "adam"):
        if not params.is_cuda or not native.available():
            raise AsyncPeerUnavailable("async xGMI exchange needs the extension and a GPU")
        if optimizer not in ("adam", "momentum", "sgd"):
            raise AsyncPeerUnavailable(f"async xGMI exchange has no '{optimizer}' update")
        P, W, r = plan.num_ps, env.world, env.rank
        for p in range(P):
            if len(plan.ps_segments(p)) != 1:
                raise AsyncPeerUnavailable("async mode needs one contiguous range per PS")
        self.plan, self.env, self.params, self.grads = plan, env, params, grads
        self.servers = servers
        self.steps = steps_per_worker
        self.grad_scale = 1.0  # the async PS applies each worker's gradient as-is
        self.opt = 0 if optimizer == "adam" else 1  # sgd: the momentum update with mu = 0
        self.mu = 0.0 if optimizer == "sgd" else None
        self.ranges: List[Tuple[int, int]] = [plan.ps_segments(p)[0] for p in range(P)]
        self.hosts = [plan.host_rank(p, W) for p in range(P)]
        ops = native.ops()

        def agree(ok: bool, why: str, what: str) -> None:
            if W == 1:
                if not ok:
                    raise AsyncPeerUnavailable(f"{what} failed: {why}")
                return
            votes = [None] * W
            dist.all_gather_object(votes, (bool(ok), why))
            bad = [(q, w) for q, (o, w) in enumerate(votes) if not o]
            if bad:
                raise AsyncPeerUnavailable(f"{what} failed on ranks {bad}")

        peer, mine, why = None, None, ""
        try:
            peer = ops.AsyncPeer(params, grads, W, r, [tuple(map(int, x)) for x in self.ranges],
                                 [int(h) for h in self.hosts])
            mine = peer.handle()
        except RuntimeError as e:
            why = str(e)
        agree(mine is not None, why, "async xGMI buffer export")
        handles = [mine]
        if W > 1:
            handles = [None] * W
            dist.all_gather_object(handles, mine)
        why = ""
        try:
            peer.open(handles)
        except RuntimeError as e:
            why = str(e)
        agree(not why, why, "async xGMI peer mapping")
        done_name = f"/{job_id}_xdone"
        why = ""
        try:
            if r == 0:
                peer.attach_done(done_name, True)
        except RuntimeError as e:
            why = str(e)
        agree(not why, why, "async xGMI completion counters (create)")
        try:
            if r != 0:
                peer.attach_done(done_name, False)
        except RuntimeError as e:
            why = str(e)
        agree(not why, why, "async xGMI completion counters (attach)")
        self.peer = peer
        self._selftest(agree)

        if W > 1:
            dist.barrier()
        self.coef = 1.0
        self.timeout_s = 600.0
        self._svc = None
        self.served = 0
        self.check_provenance = check_provenance
        self.provenance: List[Tuple[int, int, int, int]] = []
        self.runner = None
        self.service_mode = None
        self.inline = False
        self.inline_ok = False

    # -- the native worker step ----------------------------------------------------------------------
    def attach_runner(self, engine, segments) -> None:
        """Issue the worker step from C++ (csrc/kernels/async_runner.hip) — forward, the backward
        segments with each PS's push launched as soon as its range is complete (the push posts
        itself on the arrival board), the previous round's pull as a host wait at the start of
        the step — when the engine is the HIP one.  DDL_ASYNC_NATIVE=0 keeps the Python
        push_pull path."""
        from ..models.layout import TENSORS
        if getattr(engine, "name", "") != "hip" or os.environ.get("DDL_ASYNC_NATIVE", "1") != "1":
            return
        seg_of = {t: s for s, ts in enumerate(segments) for t in ts}
        off = self.plan.tensor_offsets
        seg_of_ps = []
        for lo, hi in self.ranges:
            ts = [t.index for t in TENSORS if off[t.index] < hi and off[t.index] + t.numel > lo]
            seg_of_ps.append(max(seg_of[t] for t in ts))
        self.runner = native.ops().AsyncRunner(engine.eng, self.peer, self.env.world,
                                               self.env.rank, seg_of_ps, self.epoch)
        # one worker hosting every PS (W = 1) with Adam: the pushes are applied in-line, as
        # tail blocks of the next backward launch (async_runner.hip set_inline); start() turns
        # it on once the PS state is final (a resume loads it after this point).
        # DDL_ASYNC_INLINE=0 keeps the push / board / apply / gate chain at W = 1.
        self.inline_ok = (self.env.world == 1 and self.opt == 0
                          and os.environ.get("DDL_ASYNC_INLINE", "1") == "1")

    def native_step(self, engine, x, y, keep_prob: float, seed: int) -> None:
        engine._set_keep(keep_prob)
        self.runner.step(x if x.is_contiguous() else x.contiguous(), y, seed & 0xFFFFFFFF,
                         self.timeout_s)
        self.epoch += 1

    def drain_round(self) -> None:
        """The round in flight (native step) has come back: this worker's parameters are final
        until its next step (checkpoint hook)."""
        if self.runner is not None:
            self.runner.finish(self.timeout_s)
            if self.inline:  # the PS private copies follow the worker buffer they equal
                self.runner.inline_sync_ps()
                torch.cuda.synchronize(self.params.device)

    # -- set-up check ------------------------------------------------------------------------------
    def _selftest(self, agree) -> None:
        """Round 1 with the self-test update (PS shard := pushed gradient): every worker must
        get back exactly what it pushed, from every PS."""
        W, r = self.env.world, self.env.rank
        dev = self.params.device
        saved = self.params.clone()
        n = self.params.numel()
        pat = (torch.arange(n, device=dev) % 13 + 1).to(torch.float32) * float(r + 1)
        self.grads.copy_(pat)
        self.params.zero_()
        torch.cuda.synchronize(dev)
        self.peer.push_all(1, 1.0)
        torch.cuda.synchronize(dev)
        if W > 1:
            dist.barrier()  # every push has completed before any apply is issued
        for p, (lo, hi) in enumerate(self.ranges):
            if self.hosts[p] != r:
                continue
            tmp = torch.empty(hi - lo, device=dev)
            for w in range(W):
                self.peer.apply(p, w, 1, 2, tmp, None, None, 0.0, 0.9, 0.999, 1e-8, 0.0, 0.0, 1.0)
        ok = self.peer.wait_done(1, 60.0)
        torch.cuda.synchronize(dev)
        why = f"timed out (code {self.peer.error()})"
        ok = ok and self.peer.error() == 0
        if ok:
            for lo, hi in self.ranges:
                if not torch.equal(self.params[lo:hi], pat[lo:hi]):
                    bad = int((self.params[lo:hi] != pat[lo:hi]).nonzero()[0]) + lo
                    ok, why = False, f"mismatch at {bad}"
                    break
        self.params.copy_(saved)
        self.grads.zero_()
        torch.cuda.synchronize(dev)
        agree(ok, why, "async xGMI self-test")
        self.epoch = 1                                   # worker rounds done

    # -- PS service thread -------------------------------------------------------------------------
    def _expected(self) -> int:
        W, r = self.env.world, self.env.rank
        return sum(1 for h in self.hosts if h == r) * W * self.steps

    def start(self) -> None:
        """The service loop in C++ (xgmi_async.hip AsyncService): no Python and no GIL between
        a remote worker's push and its apply kernel."""
        n = self._expected()
        if n == 0:
            return
        ps_list = [(p, ps.params, ps.m, ps.v, ps.t) for p, ps in self.servers.items()]
        h = next(iter(self.servers.values())).h
        if self.runner is not None and self.inline_ok and len(ps_list) == self.plan.num_ps and \
                all(torch.equal(ps.params, self.params[lo:hi])
                    for p, ps in self.servers.items() for lo, hi in [self.ranges[p]]):
            # (a PS that does not start from the worker's parameters — --ref-quirks Q4 — keeps
            # the service: its apply stores the PS copy into the worker buffer)
            self.runner.set_inline(ps_list, h.lr, h.beta1, h.beta2, h.eps, self.grad_scale,
                                   self.check_provenance)
            self.inline = True
            self._inline_t0 = {p: ps.t for p, ps in self.servers.items()}
            self.service_mode = "inline"
            return
        mom = next(iter(self.servers.values())).momentum if self.mu is None else self.mu
        self._svc = native.ops().AsyncService(
            self.peer, self.env.world, ps_list, self.opt, h.lr, h.beta1, h.beta2, h.eps, mom,
            self.grad_scale, 1, self.check_provenance)
        self._svc.start(n)
        self.service_mode = self._svc.mode()  # "host": the native board-scan service

    def _sync_counters(self, svc) -> None:
        """The native service advances each hosted PS's step counter; mirror it into the
        Python ParameterServer objects (checkpoints and reports read those)."""
        for p, ps in self.servers.items():
            n = svc.t(p) - ps.t
            ps.t += n
            ps.updates += n

    def _sync_inline(self) -> None:
        """In-line applies: the runner holds the step counters and the worker buffer holds the
        parameters (drain_round wrote them back into the PS objects' private copies)."""
        self._sync_counters(_RunnerCounters(self.runner))

    @contextlib.contextmanager
    def paused(self):
        """Checkpoint hook: no PS update is issued inside the block and every issued one has
        completed, so each hosted PS's parameters, m, v and t are one consistent step."""
        if self.inline:  # every apply is on this worker's stream: drained by drain_round
            self.drain_round()
            self._sync_inline()
            yield
            return
        svc = self._svc
        if svc is None:  # not started (or joined): no update in flight
            yield
            return
        svc.pause()
        try:
            self._sync_counters(svc)
            yield
        finally:
            svc.resume()

    def join(self) -> None:
        self.drain_round()  # this worker's last round (the reference's final pull)
        if self.inline:
            self._sync_inline()
            self.served = sum(self.runner.inline_t(p) - t0 for p, t0 in self._inline_t0.items())
            if self.check_provenance:
                self.provenance = [(w, p, e - 2, t)
                                   for (w, p, e, t) in self.runner.inline_provenance()]
        if self._svc is not None:
            svc, self._svc = self._svc, None
            try:
                svc.join()
            finally:
                self._sync_counters(svc)
                self.served = svc.served()
                if self.check_provenance:
                    self.provenance = [(w, p, e - 2, t) for (w, p, e, t) in svc.provenance()]
        if self.peer.error():
            raise RuntimeError(f"async xGMI wait timed out (code {self.peer.error()})")

    def verify_provenance(self) -> None:
        """Every hosted PS applied exactly `steps` pushes of every worker, in step order, and
        its step counter advanced once per push."""
        for p in self.servers:
            for w in range(self.env.world):
                steps = [s for (ww, pp, s, _) in self.provenance if ww == w and pp == p]
                if steps != list(range(self.steps)):
                    raise RuntimeError(f"provenance: PS {p} / worker {w} steps {steps[:5]}...")
            ts = [t for (_, pp, _, t) in self.provenance if pp == p]
            if ts != sorted(ts) or len(set(ts)) != len(ts):
                raise RuntimeError(f"provenance: PS {p} step counter not strictly increasing")

    # -- worker side --------------------------------------------------------------------------------
    def push_pull(self) -> None:
        """Push round e (posted on the board by the kernel), wait until every PS stored the
        parameters back (host-side: the reference's blocking pull)."""
        self.epoch += 1
        self.peer.push_all(self.epoch, self.coef)
        if not self.peer.wait_done(self.epoch, self.timeout_s):
            raise RuntimeError(f"async xGMI: round {self.epoch} did not come back "
                               f"(kernel error code {self.peer.error()})")

    def close(self) -> None:
        """Release the data plane deterministically (every rank, same program point, after
        join()): the service's stream, the peer mappings, inbox / flags and the shm board."""
        if self._svc is not None:  # a run that never joined (error path)
            svc, self._svc = self._svc, None
            svc.join()
        self.runner = None
        if self.peer is not None:
            self.peer.close()
