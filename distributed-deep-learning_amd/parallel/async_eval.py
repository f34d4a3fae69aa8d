"""Evaluation off the training stream: the reference's every-10-steps test-set eval
(``mnist_sync/worker.py:71-72``) from a parameter snapshot, on a side HIP stream.

The reference evaluates in line: ``sess.run(accuracy)`` blocks the worker, and the full 10k
test-set forward (0.71 TFLOP, 3.3x the FLOPs of the 10 training steps between evals) is most
of the time to a target accuracy.  Here the training stream only copies the parameters into a
snapshot slot (10 MB, a few us) and records an event; a second stream waits for that event,
copies the slot into the eval engine's own parameter buffer and runs the large-M eval GEMMs
while the training stream's latency-bound small GEMMs keep going.  The training stream never
waits on the eval stream (except to reuse a snapshot slot still unread, which needs more than
``slots`` evals in flight).  Accuracy semantics are unchanged — eval i scores exactly the
parameters after step i — and the time to a target accuracy is the GPU time at which that
eval's result exists (events on the eval stream vs one on the training stream at the start).

Measured (bench.py time-to-95 %, one MI355X): 0.200 s in line -> 0.185-0.188 s; the eval's
0.71 TFLOP per pass still dominates (the GPU is nearly saturated by it), so the overlap hides
the training steps' idle gaps rather than the eval.  ``DDL_EVAL_CHUNK`` sets the eval engine's
rows per forward (10k default; 2k measured the same, 1k slower).

W > 1 (sync, ``dist_eval``): each rank scores its 1/W slice; the counts and completion times
are combined with one all-reduce (sum / max) at ``drain``, so the eval lines print then.
"""
from __future__ import annotations

import os
from collections import deque
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

Result = Callable[[dict, float, float], None]  # (meta, accuracy, seconds since start)


class AsyncEvaluator:
    def __init__(self, trainer, on_result: Optional[Result] = None, slots: int = 64):
        from ..models.hip_engine import HipEngine
        tr = trainer
        self.tr = tr
        self.on_result = on_result
        dev = tr.params.device
        # Stream priorities.  torch's HIP stream pool offers priorities <= 0 only (a positive
        # request maps to 0), so "low" does not exist here: the eval stream and the training
        # stream are both NORMAL priority (0) and share the normal hardware-queue pool (a HIGH
        # priority eval stream measured the same time to 95 %: 0.1404-0.1417 vs 0.1415-0.1422 s,
        # profiles/r3_ab_evalprio.log).
        # The training stream is NORMAL priority in both modes: the native runners' GPU-side
        # gates rely on the training (compute) stream never sharing a hardware queue with their
        # high-priority comm / PS-service streams, and HIP pools hardware queues per priority
        # (runner.hip, async_runner.hip; a high-priority training stream stalled the W = 2
        # one-card time-to-accuracy run).
        # (torch's pooled streams: the pool is fixed per device and priority, so evaluators
        # built one after another reuse the same streams and hardware queues; destroying an
        # external stream instead left the caching allocator's blocks tied to a dead stream)
        self.stream = torch.cuda.Stream(device=dev, priority=0)
        self.train_stream = torch.cuda.Stream(device=dev, priority=0)
        self.snap = torch.empty_like(tr.params)
        chunk = int(os.environ.get("DDL_EVAL_CHUNK", "10000"))
        self.engine = HipEngine(self.snap, torch.zeros_like(tr.params), tr.plan.tensor_offsets,
                                batch=tr.cfg.batch_size, graph=False, eval_chunk=chunk)
        env = tr.env
        x, y = tr.data.x_test, tr.data.y_test
        n = x.shape[0]
        self.n_test = n
        self.dist = tr.cfg.dist_eval and tr.cfg.mode == "sync" and env.world > 1
        if self.dist:
            per = (n + env.world - 1) // env.world
            lo, hi = min(n, env.rank * per), min(n, (env.rank + 1) * per)
            x, y = x[lo:hi], y[lo:hi]
        self.x, self.y = x, y
        self.slots = slots
        self.ring: List[Optional[torch.Tensor]] = [None] * slots
        self.host = torch.zeros(slots, dtype=torch.int32, pin_memory=True)
        self.busy = [None] * slots          # pending record using the slot
        self.pending: deque = deque()
        self.done_records: List[dict] = []  # finished (meta, count, ms) in submit order
        self.t0 = torch.cuda.Event(enable_timing=True)
        self.n = 0

    def close(self) -> None:
        """Drop the eval engine (its 10k-row workspace, ~2.6 GB) and the snapshot ring now,
        after the last eval, instead of whenever garbage collection gets to them."""
        if self.engine is None:
            return
        self.drain()
        torch.cuda.current_stream().wait_stream(self.train_stream)
        torch.cuda.synchronize()
        self.engine = None
        self.ring = [None] * self.slots
        self.snap = None

    def start(self) -> None:
        """Time origin: recorded on the training stream when the training clock starts."""
        self.t0.record()

    def submit(self, meta: dict) -> None:
        j = self.n % self.slots
        self.n += 1
        if self.busy[j] is not None:  # slot still read by an unfinished eval: wait for it
            self.busy[j]["done"].synchronize()
            self.poll()
        if self.ring[j] is None:
            self.ring[j] = torch.empty_like(self.tr.params)
        slot = self.ring[j]
        slot.copy_(self.tr.params)  # training stream: parameters after this step
        ev = torch.cuda.Event()
        ev.record()
        rec = dict(meta=meta, slot=j, done=torch.cuda.Event(enable_timing=True))
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            self.snap.copy_(slot)
            cnt = self.engine.correct_async(self.x, self.y)
            self.host[j:j + 1].copy_(cnt, non_blocking=True)
            rec["done"].record(self.stream)
        self.busy[j] = rec
        self.pending.append(rec)

    def _finish(self, rec) -> None:
        j = rec["slot"]
        rec["count"] = int(self.host[j])
        rec["ms"] = self.t0.elapsed_time(rec["done"])
        self.busy[j] = None
        self.done_records.append(rec)

    def poll(self) -> None:
        """Finish every eval whose result exists (in submit order, no host sync); without
        dist eval report it at once: on_result(meta, acc, seconds since start)."""
        on_result = self.on_result
        while self.pending and self.pending[0]["done"].query():
            rec = self.pending.popleft()
            self._finish(rec)
            if not self.dist:
                self.done_records.pop()
                if on_result is not None:
                    on_result(rec["meta"], rec["count"] / self.n_test, rec["ms"] / 1e3)

    def drain(self) -> None:
        """Wait for every submitted eval; with dist eval combine the ranks' counts (sum) and
        completion times (max) and report all results in order."""
        on_result = self.on_result
        self.stream.synchronize()
        self.poll()
        if not self.dist:
            return
        recs, self.done_records = self.done_records, []
        if not recs:
            return
        dev = self.tr.params.device
        counts = torch.tensor([r["count"] for r in recs], dtype=torch.float64, device=dev)
        times = torch.tensor([r["ms"] for r in recs], dtype=torch.float64, device=dev)
        dist.all_reduce(counts)
        dist.all_reduce(times, op=dist.ReduceOp.MAX)
        if on_result is not None:
            for r, c, t in zip(recs, counts.tolist(), times.tolist()):
                on_result(r["meta"], c / self.n_test, t / 1e3)
