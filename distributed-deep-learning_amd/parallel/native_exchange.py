"""Native synchronous exchange: the whole sync training step in the C++ ``SyncRunner``.

Same plan and the same units as :class:`~.comm.SyncExchange` (whose planner this reuses);
the per-step work — forward, the four backward segments, and per unit
reduce-scatter/Adam/all-gather (flat plan) or reduce/Adam/broadcast (tensor-granular plans)
or a local Adam (W = 1) — is enqueued by ``csrc/kernels/runner.hip`` in one call, on a
high-priority comm stream that waits per backward segment.  The Python exchange spends
tens of microseconds of host time per collective and per update, which left the GPU idle
at every segment boundary; here the host issues the step in ~one launch per kernel.

RCCL: the runner owns its own communicator on torch's librccl instance; the unique id is
broadcast over the default process group.  Before the native path is trusted on a
multi-GPU job, a collective self-test (reduce-scatter/all-gather and reduce/broadcast on a
known pattern) runs on every rank and the decision to use it is agreed by all ranks.
PS state (``m``/``v``/step counter ``t``) stays in the Python ``ParameterServer`` objects, so
checkpointing and inspection are unchanged.

``backend="xgmi"``: instead of RCCL, each bucket is ONE fused kernel over IPC-mapped peer memory
(``csrc/kernels/xgmi.hip``): push the gradients to their owners, owner sum + optimizer, push the
parameters back.  Flat plan with one PS per GPU: equal-chunk buckets (rank r owns chunk r, the
reduce-scatter form).  Every other plan — the reference's tensor-granular ``none`` (1 PS + W
workers, ``mnist_sync/``), ``contiguous`` and ``greedy`` (``mnist_sync_sharding*/``), ``lpt``, or
a flat plan with fewer PS than GPUs — gets one OWNER bucket per exchange unit (one PS's tensors
completed by one backward segment): every rank pushes the unit to the rank hosting that PS, which
sums, updates with the PS's state and pushes the parameters to every rank.  Set up collectively
(IPC handles all-gathered over the default group) and verified by a self-test on a known pattern
whose result all ranks vote on; it needs no RCCL communicator, so it also runs with several ranks
on ONE GPU (gloo default group) — the multi-process rehearsal of the W > 1 step on a one-GPU box.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, Sequence

import torch
import torch.distributed as dist

from ..ops import native
from ..ops.adam import adam_coeffs
from .comm import DistEnv, SyncExchange
from .ps import ParameterServer
from .sharding import ShardPlan

_KIND = {"local": 0, "rs": 1, "reduce": 2, "xgmi": 3, "ar": 4, "xgmi_repl": 5}


class NativeUnavailable(RuntimeError):
    pass


def last_segment_bucket(plan: ShardPlan, segments: Sequence[Sequence[int]]) -> int:
    """Index of the bucket whose gradients complete LAST (the final backward segment's).

    ``make_plan`` orders buckets by their smallest tensor id, so for the HIP engine's segments
    ([fc], [conv4], [conv3], [conv2 + conv1]) the last-completed bucket is bucket 0, not the
    last index: replicating ``len - 1`` (round 3) replicated the 1.58 M-parameter fc bucket —
    the FIRST to complete, on the comm stream, with no DONE words for the final wait to see —
    instead of the 52 k-parameter conv1 + conv2 bucket on the step's exposed end."""
    last = set(int(t) for t in segments[-1])
    buckets = plan.meta.get("buckets") or []
    holders = [i for i, bk in enumerate(buckets) if last <= set(bk)]
    if len(holders) != 1:
        raise NativeUnavailable("flat plan buckets do not match the engine's segments")
    b = holders[0]  # (an unbucketed plan, no overlap: the one bucket of every tensor)
    lo, hi = plan.bucket_ranges[b]
    offs = plan.tensor_offsets
    from ..models.layout import TENSORS
    want_lo = min(offs[t] for t in last)
    want_hi = max(offs[t] + TENSORS[t].numel for t in last)
    assert lo <= want_lo and want_hi <= hi, (b, (lo, hi), (want_lo, want_hi))
    return b


class NativeSyncExchange(SyncExchange):
    native = True
    uses_side = False  # collectives go on the C++ runner's own comm stream

    def __init__(self, plan: ShardPlan, env: DistEnv, params: torch.Tensor, grads: torch.Tensor,
                 segments: Sequence[Sequence[int]], servers: Dict[int, ParameterServer], engine,
                 grad_reduce: str = "sum", ref_quirks: bool = False, overlap: bool = True,
                 optimizer: str = "adam", hyper=None, momentum: float = 0.9,
                 force_collectives: bool = False, backend: str = "rccl"):
        if optimizer not in ("adam", "momentum", "sgd"):
            raise NativeUnavailable(f"native runner has no '{optimizer}' update")
        if optimizer == "sgd":
            # plain SGD = the fused momentum kernel with mu = 0 (m holds the last gradient)
            momentum = 0.0
        if not params.is_cuda or getattr(engine, "name", "") != "hip":
            raise NativeUnavailable("native runner needs the HIP engine on a GPU")
        if len(segments) != 4:
            raise NativeUnavailable("native runner expects the engine's 4 backward segments")
        super().__init__(plan, env, params, grads, segments, servers, grad_reduce, ref_quirks,
                         overlap=overlap, force_collectives=force_collectives)
        self.engine = engine
        self.optimizer = optimizer
        ops = native.ops()
        # The step's LAST bucket (conv2 + conv1, 52 k parameters) completes with the backward, so
        # nothing overlaps its exchange.  Replicate its update: one all-reduce (RCCL) or one
        # all-to-all push (xGMI) of the whole bucket, every rank sums in rank order and runs the
        # optimizer on replicated state — one hop on the exposed end of the step instead of
        # reduce-scatter -> owner update -> all-gather.  The PS objects keep their chunk of that
        # state for checkpoints (sync_ps_state / load_ps_state).  DDL_REPL_LAST=0: owner form.
        self.repl = None
        if (self.collective and plan.bucket_ranges is not None and plan.num_ps == env.world
                and os.environ.get("DDL_REPL_LAST", "1") == "1"):
            b = last_segment_bucket(plan, segments)
            lo, hi = plan.bucket_ranges[b]
            z = lambda: torch.zeros(hi - lo, dtype=torch.float32, device=params.device)  # noqa: E731
            self.repl = (b, int(lo), int(hi), z(), z() if optimizer == "adam" else None)
        self.runner = ops.SyncRunner(engine.eng, params, grads, env.world, env.rank)
        # DDL_READY_FLAGS: the comm stream's hand-off (2: READY flags for every segment, the
        # default; 1: all but the first; 0: events) — runner.hip SyncRunner::set_ready_flags
        rf = os.environ.get("DDL_READY_FLAGS")
        if rf is not None:
            self.runner.set_ready_flags(int(rf))
        self.backend = "local" if env.world == 1 and not force_collectives else backend
        self.peer = None
        self._xbucket = {}  # id(unit) -> its xGMI owner bucket (tensor-granular plans)
        if backend == "xgmi" and (env.world > 1 or force_collectives):
            # (W = 1 with force_collectives: the whole W > 1 step structure — comm stream,
            # events, fused bucket kernels, final wait — on one GPU, every push to itself)
            specs = None
            if plan.bucket_ranges is None or plan.num_ps != env.world:
                specs = self._owner_specs()
            self._init_peer_collectively(ops, env, plan, params, grads, specs)
        elif env.world > 1:
            self._init_comm_collectively(ops, env)
        elif force_collectives:
            self.runner.init_comm(ops.SyncRunner.unique_id(), True)
            ok, why = self.runner.selftest()
            if not ok:
                raise RuntimeError(f"RCCL 1-rank self-test failed: {why}")
        seg_sets = [set(s) for s in segments]
        # issue_after[s]: the backward segment after which segment s's units are issued.
        # Every issue point costs an event record on the compute stream (~4.5 us gap,
        # forced-rehearsal timeline), so the RCCL path issues the fc bucket together with conv4's
        # after segment 1 (still overlapped by the conv3 + conv2 backward): forced 1-rank
        # rehearsal 0.405 -> 0.3965 ms/step.  The xGMI kernels are one launch per bucket with no
        # ring passes, and measured 0.402 (own point) vs 0.404 (merged): each bucket right after
        # its own segment.
        issue_after = list(range(len(seg_sets)))
        if self.backend == "rccl" and len(seg_sets) == 4:
            issue_after = [1, 1, 2, 3]

        def seg_of(tensors):
            if not overlap:
                return len(seg_sets) - 1
            return issue_after[max(next(i for i, s in enumerate(seg_sets) if t in s)
                                   for t in tensors)]

        units = []
        for u in self.units:
            ps = env.rank if u.kind == "rs" else u.ps
            srv = servers.get(ps)
            offs = u.state_offs or [0] * len(u.ranges)
            ranges = [(int(lo), int(hi), int(off)) for (lo, hi), off in zip(u.ranges, offs)]
            kind = "xgmi" if (self.peer is not None and u.kind in ("rs", "reduce")) else u.kind
            m = srv.m if srv is not None else None
            v = srv.v if srv is not None else None
            shard = None if kind == "xgmi" else u.shard_buf
            bucket = self._xbucket.get(id(u), u.bucket)
            if self.repl is not None and u.kind == "rs" and u.bucket == self.repl[0]:
                kind = "xgmi_repl" if self.peer is not None else "ar"
                _, lo, hi, m, v = self.repl
                ranges, shard = [(lo, hi, 0)], None
            units.append((seg_of(u.tensors), _KIND[kind], int(u.host), int(ps), ranges,
                          m, v, shard, int(bucket)))
        h = hyper if hyper is not None else next(iter(servers.values())).h
        # (before set_units: it checks each unit's optimizer state against the update kind)
        self.runner.set_optimizer(0 if optimizer == "adam" else 1, h.lr, h.beta1, h.beta2, h.eps,
                                  momentum)
        self.runner.set_units(units)
        self.runner.set_scale(self.grad_scale, self.coef)
        # A/B knob: DDL_LAST_ON_MAIN=0 puts the last segment's collectives back on the comm
        # stream (one event hop more on the critical path of every W > 1 step)
        self.runner.set_last_on_main(os.environ.get("DDL_LAST_ON_MAIN", "1") != "0")
        self._lr = [0.0] * max(plan.num_ps, env.world)
        self._n = 0

    def _init_comm_collectively(self, ops, env: DistEnv) -> None:
        """Every go/no-go decision is voted on over the default process group BEFORE any rank
        enters a blocking RCCL call, so a rank that cannot use the native path makes all ranks
        fall back together instead of leaving the others stuck in ``ncclCommInitRank``."""
        def agree(ok: bool, why: str, what: str) -> None:
            votes = [None] * env.world
            dist.all_gather_object(votes, (bool(ok), why))
            bad = [(r, w) for r, (o, w) in enumerate(votes) if not o]
            if bad:
                raise NativeUnavailable(f"{what} failed on ranks {bad}")

        why = ops.SyncRunner.probe()
        agree(not why, why, "RCCL symbol probe")
        ids = [None, ""]
        if env.rank == 0:
            try:
                ids[0] = ops.SyncRunner.unique_id()
            except RuntimeError as e:
                ids[1] = str(e)
        dist.broadcast_object_list(ids, src=0)
        if ids[0] is None:
            raise NativeUnavailable(f"ncclGetUniqueId failed on rank 0: {ids[1]}")
        self.runner.init_comm(ids[0])
        ok, why = self.runner.selftest()
        agree(ok, why, "RCCL self-test")

    def _owner_specs(self):
        """One xGMI owner bucket per exchange unit of a plan without one equal chunk per rank:
        (runs, the runs' offsets in the owning PS's optimizer state, the hosting rank)."""
        specs = []
        for u in self.units:
            if u.kind != "reduce":
                raise NativeUnavailable(f"xgmi exchange: unexpected unit kind {u.kind}")
            if len(u.ranges) > 8:
                raise NativeUnavailable("xgmi exchange: a unit with more than 8 runs")
            offs = u.state_offs or [0] * len(u.ranges)
            self._xbucket[id(u)] = len(specs)
            specs.append(([(int(lo), int(hi)) for lo, hi in u.ranges], [int(o) for o in offs],
                          int(u.host)))
        if len(specs) > 32:
            raise NativeUnavailable(f"xgmi exchange: {len(specs)} units (at most 32)")
        return specs

    def _init_peer_collectively(self, ops, env: DistEnv, plan: ShardPlan, params: torch.Tensor,
                                grads: torch.Tensor, specs=None) -> None:
        """IPC handles out and in, then a self-test: every rank fills its gradients with
        (rank + 1) * (i % 13 + 1), one exchange with w := sum of g must give
        W (W + 1) / 2 * (i % 13 + 1) everywhere (exact in fp32).  Every stage is voted on, so
        a failure anywhere makes all ranks fall back together."""
        def agree(ok: bool, why: str, what: str) -> None:
            if env.world == 1:
                if not ok:
                    raise NativeUnavailable(f"{what} failed: {why}")
                return
            votes = [None] * env.world
            dist.all_gather_object(votes, (bool(ok), why))
            bad = [(r, w) for r, (o, w) in enumerate(votes) if not o]
            if bad:
                raise NativeUnavailable(f"{what} failed on ranks {bad}")

        peer, why = None, ""
        try:
            # at most this many workgroups per bucket kernel (>= 1024 elements each;
            # DDL_XGMI_SLICES): forced W = 1 rehearsal, round 4: 128 -> 256 -> 384: 0.3288 ->
            # 0.3243 -> 0.3230 ms/step (fewer: 64 0.331, 32 0.42 — the bucket kernels outlast
            # the backward); round 6, with the shorter duals: 160 / 192 / 224 / 256 / 384:
            # 0.2747-0.2751 / 0.2745 / 0.2759-0.2760 / 0.2774-0.2778 / 0.2784-0.2798 (the
            # high-priority bucket kernel takes fewer of the slots the duals free,
            # profiles/r6_xgmi_slices.log).  Ranks sharing one GPU (the one-box rehearsals)
            # keep 128: their spinning bucket kernels must all find room on the one card.
            shared_gpu = env.world > max(1, torch.cuda.device_count())
            slices = int(os.environ.get("DDL_XGMI_SLICES", "128" if shared_gpu else "192"))
            buckets = (specs if specs is not None
                       else [tuple(map(int, b)) for b in plan.bucket_ranges])
            peer = ops.PeerExchange(params, grads, env.world, env.rank, buckets, slices,
                                    self.repl[0] if self.repl is not None else -1)
            mine = peer.handle()
        except (RuntimeError, ValueError) as e:  # (pybind11: invalid_argument -> ValueError)
            mine, why = None, str(e)
        agree(mine is not None, why, "xGMI buffer export")
        handles = [mine]
        if env.world > 1:
            handles = [None] * env.world
            dist.all_gather_object(handles, mine)
        try:
            peer.open(handles)
            why = ""
        except (RuntimeError, ValueError) as e:
            why = str(e)
        agree(not why, why, "xGMI peer mapping")
        self.runner.set_peer(peer)
        self.peer = peer
        saved = params.clone()
        n = params.numel()
        i = torch.arange(n, device=params.device)
        pat = (i % 13 + 1).to(torch.float32)
        grads.copy_(pat * float(env.rank + 1))
        want = pat * float(env.world * (env.world + 1) // 2)
        # The stale-L2 probe (must stay: it is the one check between a real node and silent
        # replica drift).  Peers store the new parameters into this GPU's HBM over xGMI; none of
        # those stores passes through this GPU's per-XCD L2s, and the protocol relies on the next
        # kernel's start-of-kernel acquire to drop any line cached before the exchange
        # (xgmi.hip header).  So before the exchange EVERY XCD reads (caches) EVERY parameter
        # line, and after it every XCD compares every line with the expected sums: a line served
        # stale from some XCD's L2 counts as a mismatch (ops.xcd_sweep, xgmi.hip).
        probe = torch.zeros(2, dtype=torch.int32, device=params.device)
        ops.xcd_sweep(params, None, probe)
        torch.cuda.synchronize(params.device)
        self.runner.peer_selftest_step()
        ok, why = True, ""
        if not peer.error():
            ops.xcd_sweep(params, want, probe)
            torch.cuda.synchronize(params.device)
        if peer.error():
            ok, why = False, f"timed out (code {peer.error()})"
        elif int(probe[0].item()) != 0:
            ok, why = False, (f"{int(probe[0].item())} stale parameter reads across the XCDs "
                              f"after the exchange (L2 not invalidated)")
        else:
            spans = ([r for runs, _, _ in specs for r in runs] if specs is not None
                     else plan.bucket_ranges)
            for lo, hi in spans:
                if not torch.equal(params[lo:hi], want[lo:hi]):
                    bad = int((params[lo:hi] != want[lo:hi]).nonzero()[0]) + lo
                    ok, why = False, f"mismatch at {bad}: {float(params[bad])} != {float(want[bad])}"
                    break
        params.copy_(saved)
        grads.zero_()
        torch.cuda.synchronize(params.device)
        agree(ok, why, "xGMI self-test")

    def step(self, x: torch.Tensor, labels: torch.Tensor, keep_prob: float, seed: int) -> None:
        """One synchronous global step: every hosted PS advances its step counter (one
        ``apply_gradients`` per global step, like the reference PS) and the runner enqueues
        compute + exchange + update."""
        eng = self.engine
        eng._set_keep(keep_prob)
        lr = self._lr
        for p, ps in self.servers.items():
            ps.begin()
            lr[p] = adam_coeffs(ps.h, ps.t) if self.optimizer == "adam" else ps.h.lr
        self.runner.step(x if x.is_contiguous() else x.contiguous(), labels, seed & 0xFFFFFFFF, lr)
        self._n += 1
        if self.env.world > 1 and self._n % 64 == 0:
            self.check()

    # -- the READY-flag hand-off, proven per job ------------------------------
    def _snapshot(self):
        srv = {p: (ps.m.clone(), None if ps.v is None else ps.v.clone(), ps.t, ps.updates)
               for p, ps in self.servers.items()}
        repl = None if self.repl is None else tuple(
            None if x is None else x.clone() for x in self.repl[3:])
        return self.params.clone(), srv, repl

    def _restore(self, snap) -> None:
        params, srv, repl = snap
        self.params.copy_(params)
        for p, (m, v, t, n) in srv.items():
            ps = self.servers[p]
            ps.m.copy_(m)
            if v is not None:
                ps.v.copy_(v)
            ps.t, ps.updates = t, n
        if repl is not None:
            for dst, src in zip(self.repl[3:], repl):
                if dst is not None:
                    dst.copy_(src)
        torch.cuda.synchronize(self.params.device)

    def handoff_check(self, trainer, steps: int = 6, _perturb_rank=None) -> dict:
        """Prove the READY-flag hand-off on THIS job before trusting it.

        The comm stream's exchange of segment s starts behind a READY flag that the next
        segment's first launch stores (runner.hip), not behind an event with a system-scope
        release; that peers read the gradients and parameters coherently then rests on the
        kernel-boundary L2 write-back, which no single-card test can exercise.  So: from the same
        state, ``steps`` steps with the event hand-off (system fence) and ``steps`` steps with
        the READY flags, a SHA-256 of the resulting parameters on every rank; the flags are kept
        only if both modes give the same bits and every rank agrees, otherwise every rank falls
        back to the events.  If the ranks' digests disagree under the EVENT hand-off too, the
        replicas have diverged — not a hand-off-ordering problem, so events cannot repair it:
        every rank raises NativeUnavailable and the job refuses this data plane
        (``handoff_vote``).  The state (parameters, PS m / v / t, replicated state) is restored
        afterwards — with the trainer's global step (its dropout seeds) — so the caller's run
        starts where it would have."""
        import hashlib
        if self.backend == "local":
            return {"handoff": "none (every update local)"}
        snap = self._snapshot()
        g0 = trainer.global_step
        digests = {}
        try:
            for mode, rf in (("events", 0), ("ready_flags", 2)):
                self._restore(snap)
                trainer.global_step = g0
                self.runner.set_ready_flags(rf)
                for i in range(steps):
                    trainer.train_step(i)
                torch.cuda.synchronize(self.params.device)
                self.check()
                digests[mode] = hashlib.sha256(
                    self.params.detach().cpu().numpy().tobytes()).hexdigest()
        finally:
            self._restore(snap)
            trainer.global_step = g0
        if _perturb_rank is not None and self.env.rank == _perturb_rank:  # (test hook)
            digests = {k: "0" * 64 for k in digests}
        v = handoff_vote(self.env, digests["events"], digests["ready_flags"])
        forced = os.environ.get("DDL_READY_FLAGS")  # an explicit choice stays in force
        self.runner.set_ready_flags(int(forced) if forced is not None else (2 if v["ok"] else 0))
        return {"handoff": ("ready_flags" if v["ok"] else "events (READY flags failed the check)")
                + (f" (DDL_READY_FLAGS={forced} in force)" if forced is not None else ""),
                "check_steps": steps, "modes_bit_identical": v["modes_agree"],
                "ranks_bit_identical": v["ranks_agree"],
                "params_sha256": digests["ready_flags"][:16]}

    # -- replicated last bucket <-> the PS objects (checkpoint / resume) ---------------------------
    def _repl_chunk(self):
        b, lo, hi, m, v = self.repl
        r, W = self.env.rank, self.env.world
        c = (hi - lo) // W
        ps = self.servers[r]
        off = ps.seg_off[b]
        return r, c, ps, off, m, v

    def sync_ps_state(self) -> None:
        """Copy this rank's chunk of the replicated last-bucket optimizer state into its PS
        (every rank holds the same state; the PS owns its chunk in checkpoints)."""
        if self.repl is None:
            return
        r, c, ps, off, m, v = self._repl_chunk()
        ps.m[off:off + c].copy_(m[r * c:(r + 1) * c])
        if v is not None:
            ps.v[off:off + c].copy_(v[r * c:(r + 1) * c])

    def load_ps_state(self) -> None:
        """After a resume: rebuild the replicated state from every PS's restored chunk."""
        if self.repl is None:
            return
        r, c, ps, off, m, v = self._repl_chunk()
        mine = (ps.m[off:off + c].cpu(), None if v is None else ps.v[off:off + c].cpu())
        chunks = [mine]
        if self.env.world > 1:
            chunks = [None] * self.env.world
            dist.all_gather_object(chunks, mine)
        m.copy_(torch.cat([cm for cm, _ in chunks]).to(m.device))
        if v is not None:
            v.copy_(torch.cat([cv for _, cv in chunks]).to(v.device))

    def check(self) -> None:
        """Raise if RCCL reported an asynchronous communicator error."""
        err = self.runner.async_error()
        if err:
            raise RuntimeError(f"RCCL communicator error on rank {self.env.rank}: {err}")

    def abort(self) -> None:
        """Watchdog hook: abort the communicator so blocked collectives return."""
        self.runner.abort()

    def close(self) -> None:
        """Orderly teardown (every rank, same program point): the runner's communicator, comm
        stream, events and READY flags, then the xGMI peer mappings and buffers — nothing of a
        closed exchange keeps a hardware queue or an IPC mapping until garbage collection."""
        self.runner.close()
        if self.peer is not None:
            self.peer.close()


def handoff_vote(env, digest_events: str, digest_flags: str) -> dict:
    """The collective verdict of a hand-off check (every rank calls it with its own digests of
    the same steps from the same state).

    * every rank's event-hand-off digest equal, and each rank's two modes equal: the READY flags
      are proven on this job (ok);
    * event digests equal across ranks, but the READY-flag run differs somewhere: the flags are
      what diverged, so every rank falls back to the events (not ok);
    * event digests differ across ranks: the replicas of a synchronous PS step diverged under
      the reference hand-off itself.  That is not an ordering problem — events cannot repair it
      — so every rank raises NativeUnavailable (the caller drops this data plane)."""
    votes = [(digest_events, digest_flags)]
    if env.world > 1:
        votes = [None] * env.world
        dist.all_gather_object(votes, (digest_events, digest_flags))
    events_agree = len({v[0] for v in votes}) == 1
    modes_agree = all(v[0] == v[1] for v in votes)
    ranks_agree = events_agree and len({v[1] for v in votes}) == 1
    if not events_agree:
        bad = sorted({r for r, v in enumerate(votes) if v[0] != votes[0][0]} | {0})
        raise NativeUnavailable(
            f"replicas diverge across ranks under the event hand-off (ranks {bad} disagree): "
            f"refusing this data plane")
    return {"ok": modes_agree and ranks_agree, "modes_agree": modes_agree,
            "ranks_agree": ranks_agree}


def make_sync_exchange(plan, env, params, grads, segments, servers, engine, cfg, hyper):
    """Native runner when it applies (HIP engine, sync, adam/momentum/sgd), else the Python
    exchange.  On a multi-GPU job the choice is collective (self-test votes)."""
    if cfg.native_exchange:
        try:
            backend = cfg.exchange_backend if cfg.exchange_backend != "auto" else "rccl"
            return NativeSyncExchange(plan, env, params, grads, segments, servers, engine,
                                      cfg.grad_reduce, cfg.ref_quirks, cfg.overlap,
                                      cfg.optimizer, hyper, cfg.momentum,
                                      force_collectives=cfg.force_collectives, backend=backend)
        except NativeUnavailable as e:
            if env.rank == 0 and getattr(engine, "name", "") == "hip":
                print(f"[ddl_amd] native sync runner unavailable ({e}); using the Python "
                      f"exchange", file=sys.stderr)
    return SyncExchange(plan, env, params, grads, segments, servers, cfg.grad_reduce,
                        cfg.ref_quirks, overlap=cfg.overlap)
