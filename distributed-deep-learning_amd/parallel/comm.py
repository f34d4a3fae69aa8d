"""Gradient push / parameter pull over RCCL (``torch.distributed`` backend ``nccl``).

Reference data plane: 14 host-staged MPI messages per direction per
worker step, one ``Send``/``Recv`` per tensor, tags = tensor index, blocking, with no
overlap.  MI355X-first replacement:

* every rank holds GPU-resident plan-ordered flat ``params``/``grads`` buffers;
* **sync**, ``flat`` plan with one PS per GPU: per backward bucket, one
  ``reduce_scatter`` -> fused Adam on the owned 1/W chunk -> ``all_gather``, issued on a
  side stream as soon as that bucket's gradients exist, so the exchange overlaps the
  rest of backward (SURVEY.md §5.8 bucket plan);
* **sync**, tensor-granular plans (``none``/``contiguous``/``greedy``/``lpt``): per PS
  and per ready segment, ``reduce(dst=host)`` -> Adam at the host ->
  ``broadcast(src=host)`` (reference ``mnist_sync_sharding/parameter_server.py:108-126``);
* **async**: see ``AsyncExchange``.

Gradient aggregation is a *sum* like the reference PS (``parameter_server.py:36-37``),
or a mean with ``grad_reduce='mean'`` (folded into the Adam kernel as a scale).
``ref_quirks`` reproduces the reference's buggy sums by scaling
each worker's contribution before the reduce.
"""
from __future__ import annotations

import contextlib
import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Set, Tuple

import torch
import torch.distributed as dist

from .sharding import ShardPlan
from .ps import ParameterServer
from . import mailbox as mbox


# ------------------------------------------------------------------------------------------
# process bootstrap
# ------------------------------------------------------------------------------------------
@dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    backend: Optional[str] = None
    # host-only (gloo) group for control messages that must never queue behind GPU work: with
    # an RCCL default group a collective kernel can sit on a hardware queue in front of an async
    # PS's serve / apply kernel that a peer is waiting for (checkpoint metadata in async mode)
    ctrl: Optional[object] = None

    @property
    def distributed(self) -> bool:
        return self.world > 1


def share_gpu_queue_cap(local_world: int) -> Optional[str]:
    """Ranks sharing one GPU (the one-box rehearsal): one hardware queue per process.

    HIP gives every process ``GPU_MAX_HW_QUEUES`` (4) hardware queues per priority it uses.  Four
    processes with the compute, PS comm (high priority) and side-stream eval (low priority)
    streams map more user queues than the command processor's hardware queue slots, so it
    time-slices them: a kernel spinning on a peer's flag (the xGMI pull gate, an owner bucket's
    arrival wait) then waits for the queue that holds the peer's kernel to be mapped in again —
    a runlist rotation, milliseconds.  Measured on one MI355X, W = 4 one-card time-to-accuracy
    with side-stream eval: epoch 14.87 s with the default queues, 0.98 s with one queue per
    process (`profiles/r5_w4_one_card_queues.txt`).  Must run before anything initialises HIP
    (``torch.cuda.is_available()`` does; ``device_count()`` does not).  The GPU boxes export
    ``GPU_MAX_HW_QUEUES=4`` (HIP's default) for every job, so a shared-GPU job overrides it;
    ``DDL_SHARED_GPU_HW_QUEUES`` picks another value (``keep``: leave the environment alone).
    Returns the value set."""
    want = os.environ.get("DDL_SHARED_GPU_HW_QUEUES", "1")
    if local_world <= 1 or want == "keep":
        return None
    ndev = torch.cuda.device_count()
    if ndev == 0 or local_world <= ndev:
        return None  # one process per GPU: HIP's default queues
    os.environ["GPU_MAX_HW_QUEUES"] = want
    # and the sync runner's comm stream at the LEAST priority (a pool of its own, like the
    # greatest): bucket kernels waiting on a high-priority queue slowed the other ranks' GEMMs on
    # the shared card — one-card W = 2 sync 0.89 -> 0.77-0.81 ms/step (profiles/r5_one_card_poll_prio.txt)
    os.environ.setdefault("DDL_COMM_PRIORITY", "low")
    return want


def init_distributed(device: str = "auto") -> DistEnv:
    """One process per GPU.  Reads RANK/WORLD_SIZE/LOCAL_RANK (torchrun); backend
    ``nccl`` (= RCCL on ROCm) on GPU, ``gloo`` on CPU.

    ``DDL_DIST_BACKEND`` overrides the default process group's backend, and with more ranks
    than GPUs rank ``l`` uses GPU ``l % count``: ``DDL_DIST_BACKEND=gloo`` with several ranks on
    ONE GPU is the multi-process rehearsal of a W > 1 job on a one-GPU box (RCCL refuses two
    ranks on one device; the xGMI exchange and everything above it run unchanged)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    share_gpu_queue_cap(int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
    use_gpu = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
    backend = None
    if world > 1:
        backend = os.environ.get("DDL_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        ndev = torch.cuda.device_count()
        if backend == "gloo" and ndev > 0:
            local_dev = local % ndev  # several ranks per GPU: the one-box rehearsal only
        elif local >= ndev:
            # RCCL refuses two ranks of one communicator on one device: fail here, clearly,
            # instead of with a late RCCL error or hang
            raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} GPU(s) visible: start one "
                               f"process per GPU (or DDL_DIST_BACKEND=gloo for the shared-GPU "
                               f"rehearsal)")
        else:
            local_dev = local
        torch.cuda.set_device(local_dev)
        dev = torch.device("cuda", local_dev)
    else:
        dev = torch.device("cpu")
    if world > 1:
        if not dist.is_initialized():
            kw = {}
            if use_gpu and backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    ctrl = None
    if world > 1 and backend != "gloo":
        ctrl = dist.new_group(backend="gloo")  # collective: every rank, same point
    return DistEnv(rank, world, local, dev, backend, ctrl)


def _stream_ctx(s):
    return torch.cuda.stream(s) if s is not None else contextlib.nullcontext()


# ------------------------------------------------------------------------------------------
# sync exchange
# ------------------------------------------------------------------------------------------
@dataclass
class Unit:
    kind: str                       # "rs" | "reduce" | "local"
    tensors: Set[int]
    ranges: List[Tuple[int, int]]   # plan-buffer ranges (rs: whole bucket; reduce: PS slice)
    ps: int = -1                    # reduce/local: PS id; rs: -1 (all)
    host: int = 0
    state_offs: List[int] = field(default_factory=list)
    shard_buf: Optional[torch.Tensor] = None
    bucket: int = -1                # flat plan: index into plan.bucket_ranges


def quirk_coefficient(plan: ShardPlan, rank: int, world: int, ref_quirks: bool) -> float:
    """Per-worker gradient multiplier that turns an honest sum into the reference's.

    Q1 (single sync PS, ``mnist_sync/parameter_server.py:36-37``): buffer 0 is added to
    itself -> 2*g_1 + g_2 + ... + g_W.  Q2 (sharded sync PS aliasing,
    ``mnist_sync_sharding/parameter_server.py:47,78-80``): g_last * 2**(W-1)."""
    if not ref_quirks or world == 1:
        return 1.0
    if plan.policy == "none":
        return 2.0 if rank == 0 else 1.0
    return float(2 ** (world - 1)) if rank == world - 1 else 0.0


class SyncExchange:
    uses_side = True

    def __init__(self, plan: ShardPlan, env: DistEnv, params: torch.Tensor,
                 grads: torch.Tensor, segments: Sequence[Sequence[int]],
                 servers: Dict[int, ParameterServer], grad_reduce: str = "sum",
                 ref_quirks: bool = False, overlap: bool = True, group=None,
                 force_collectives: bool = False):
        self.plan, self.env = plan, env
        # W = 1 normally updates locally; forcing keeps the collective unit kinds (run by the
        # native runner on a 1-rank RCCL communicator: the exchange path tested on one GPU)
        self.collective = env.world > 1 or force_collectives
        self.params, self.grads = params, grads
        self.servers = servers
        self.group = group
        self.world = env.world
        self.grad_scale = 1.0 / env.world if grad_reduce == "mean" else 1.0
        self.coef = quirk_coefficient(plan, env.rank, env.world, ref_quirks)
        # Without overlap every unit is issued after the whole backward (the last engine
        # segment), as one merged segment.
        self.overlap = overlap
        self.n_engine_segments = len(segments)
        self.segments = [set(s) for s in segments] if overlap else [set().union(*map(set, segments))]
        self.units = self._build_units()
        cuda = params.is_cuda
        # the Python exchange's comm stream (the native runner has its own)
        self.side = torch.cuda.Stream(device=params.device) if cuda and self.uses_side else None
        self._pending: List = []
        self._issued: Set[int] = set()
        self._ready: Set[int] = set()
        self.bytes_per_step = 4 * plan.total

    # -- planning ------------------------------------------------------------------------------
    def _build_units(self) -> List[Unit]:
        plan, W = self.plan, self.world
        units: List[Unit] = []
        tensor_of_elem = []  # (lo, hi, id) for mapping ranges -> tensors
        from ..models.layout import TENSORS
        for t in TENSORS:
            o = plan.tensor_offsets[t.index]
            tensor_of_elem.append((o, o + t.numel, t.index))

        def tensors_in(lo, hi):
            return {i for (a, b, i) in tensor_of_elem if a < hi and b > lo}

        if plan.bucket_ranges is not None:
            for bi, (lo, hi) in enumerate(plan.bucket_ranges):
                ts = tensors_in(lo, hi)
                if self.collective and plan.num_ps == W:
                    u = Unit("rs", ts, [(lo, hi)], bucket=bi)
                    c = (hi - lo) // W
                    u.shard_buf = torch.empty(c, dtype=torch.float32, device=self.params.device)
                    if self.env.rank in self.servers:
                        u.state_offs = [self.servers[self.env.rank].seg_off[bi]]
                    units.append(u)
                else:
                    for p in range(plan.num_ps):
                        seg = plan.ps_segments(p)[bi]
                        host = plan.host_rank(p, W)
                        u = Unit("reduce" if self.collective else "local", ts, [seg], p, host)
                        if p in self.servers:
                            u.state_offs = [self.servers[p].seg_off[bi]]
                        units.append(u)
            return units
        # tensor-granular: per PS, per segment, contiguous runs of that PS's tensors
        for p in range(plan.num_ps):
            host = plan.host_rank(p, W)
            mine = [i for i in plan.order if plan.owner[i] == p]
            ps_lo = plan.ps_ranges[p][0]
            for seg in self.segments:
                ids = [i for i in mine if i in seg]
                if not ids:
                    continue
                runs: List[Tuple[int, int]] = []
                for i in sorted(ids, key=lambda i: plan.tensor_offsets[i]):
                    lo, hi = plan.tensor_extent(i)  # includes alignment padding
                    if runs and runs[-1][1] == lo:
                        runs[-1] = (runs[-1][0], hi)
                    else:
                        runs.append((lo, hi))
                u = Unit("reduce" if self.collective else "local", set(ids), runs, p, host)
                u.state_offs = [lo - ps_lo for lo, _ in runs]
                units.append(u)
        return units

    # -- per step --------------------------------------------------------------------------------
    def begin_step(self) -> None:
        self._issued.clear()
        self._ready.clear()
        self._pending.clear()
        for p, ps in self.servers.items():
            ps.begin()  # one apply_gradients per global step

    def grads_ready(self, seg_index: int) -> None:
        """Called (host side, in stream order) after the engine enqueued the kernels of
        backward segment ``seg_index``."""
        if not self.overlap and seg_index < self.n_engine_segments - 1:
            return  # the merged segment is complete only after the last engine segment
        self._ready |= self.segments[min(seg_index, len(self.segments) - 1)]
        for k, u in enumerate(self.units):
            if k in self._issued or not u.tensors <= self._ready:
                continue
            self._issued.add(k)
            self._issue(u)

    def _issue(self, u: Unit) -> None:
        g, w = self.grads, self.params
        if self.coef != 1.0:
            for lo, hi in u.ranges:
                g[lo:hi].mul_(self.coef)
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream(w.device))
        with _stream_ctx(self.side):
            if u.kind == "local":
                ps = self.servers[u.ps]
                for (lo, hi), off in zip(u.ranges, u.state_offs):
                    ps.apply(w[lo:hi], g[lo:hi], off, self.grad_scale)
            elif u.kind == "rs":
                lo, hi = u.ranges[0]
                c = (hi - lo) // self.world
                r = self.env.rank
                work = dist.reduce_scatter_tensor(u.shard_buf, g[lo:hi], group=self.group,
                                                  async_op=True)
                work.wait()
                mine = w[lo + r * c: lo + (r + 1) * c]
                self.servers[r].apply(mine, u.shard_buf, u.state_offs[0], self.grad_scale)
                self._pending.append(dist.all_gather_into_tensor(w[lo:hi], mine, group=self.group,
                                                                 async_op=True))
            else:  # reduce to host, update at host, broadcast from host
                me = self.env.rank == u.host
                works = [dist.reduce(g[lo:hi], dst=u.host, group=self.group, async_op=True)
                         for lo, hi in u.ranges]
                if me:
                    for wk in works:
                        wk.wait()
                    ps = self.servers[u.ps]
                    for (lo, hi), off in zip(u.ranges, u.state_offs):
                        ps.apply(w[lo:hi], g[lo:hi], off, self.grad_scale)
                else:
                    self._pending.extend(works)
                for lo, hi in u.ranges:
                    self._pending.append(dist.broadcast(w[lo:hi], src=u.host, group=self.group,
                                                        async_op=True))

    def finish_step(self) -> None:
        if len(self._issued) != len(self.units):
            self.grads_ready(self.n_engine_segments - 1)
            # any unit still not issued covers tensors of no segment: issue now
            for k, u in enumerate(self.units):
                if k not in self._issued:
                    self._issued.add(k)
                    self._issue(u)
        with _stream_ctx(self.side):
            for wk in self._pending:
                wk.wait()
        self._pending.clear()
        if self.side is not None:
            torch.cuda.current_stream(self.params.device).wait_stream(self.side)


# ------------------------------------------------------------------------------------------
# async exchange
# ------------------------------------------------------------------------------------------
class AsyncExchange:
    """Lock-free asynchronous PS over point-to-point RCCL.

    Worker side (``push_pull``): for each PS p in order — post ``(rank, p)`` to the
    host's mailbox, ``send`` the gradient shard, ``recv`` the freshly updated parameter
    shard (reference ``mnist_async_sharding/worker.py`` Send/Recv loop).  Each worker has
    at most one push in flight per PS (staleness bound).

    PS side: one service thread per process pops arrivals in order, ``recv``s the whole
    shard gradient from that worker, applies Adam *atomically per shard* (fixing the
    reference's per-tag mixing race), and ``send``s the shard back to
    that worker.  Local pushes bypass the network under the PS lock.

    Every (worker, host) pair gets its own 2-rank communicator so the worker thread and
    the service thread never share a communicator's op order.
    """

    def __init__(self, plan: ShardPlan, env: DistEnv, params: torch.Tensor, grads: torch.Tensor,
                 servers: Dict[int, ParameterServer], steps_per_worker: int,
                 grad_reduce: str = "sum", mailbox_kind: str = "auto", job_id: str = "ddl",
                 check_provenance: bool = False):
        for p in range(plan.num_ps):
            if len(plan.ps_segments(p)) != 1:
                raise ValueError("async mode needs one contiguous range per PS "
                                 "(use a tensor-granular plan or an unbucketed flat plan)")
        if env.world > 1 and params.is_cuda and env.backend != "nccl":
            # gloo has no GPU send/recv: the RCCL pair path needs the nccl (RCCL) backend
            raise RuntimeError("async RCCL-pair exchange needs the nccl backend for GPU tensors "
                               "(with several ranks on one GPU use --exchange xgmi)")
        self.plan, self.env = plan, env
        self.params, self.grads = params, grads
        self.servers = servers
        self.steps = steps_per_worker
        self.grad_scale = 1.0  # async PS applies each worker's gradient as-is
        W, r = env.world, env.rank
        self.pair_groups: Dict[Tuple[int, int], object] = {}
        if W > 1:
            for a in range(W):
                for b in range(W):
                    if a != b:
                        g = dist.new_group([a, b])
                        if r in (a, b):
                            self.pair_groups[(a, b)] = g
        store = dist.distributed_c10d._get_default_store() if W > 1 else None
        self.mailbox = None
        if W > 1:
            hosted = [p for p in range(plan.num_ps) if plan.host_rank(p, W) == r]
            name = f"{job_id}_mbox_{r}"
            self.mailbox = mbox.make_mailbox(mailbox_kind, store, name, owner=True) if hosted else None
            dist.barrier()
            self.remote_boxes = {}
            for h in range(W):
                if h != r and any(plan.host_rank(p, W) == h for p in range(plan.num_ps)):
                    self.remote_boxes[h] = mbox.make_mailbox(mailbox_kind, store, f"{job_id}_mbox_{h}",
                                                             owner=False)
        for ps in servers.values():
            ps.gbuf = torch.empty(ps.numel, dtype=torch.float32, device=params.device)
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self.served = 0
        # Race detection: with check_provenance every push carries a
        # (step, fp64 checksum) header; the PS verifies that the bytes it applies are exactly
        # what that worker pushed for that step, that each worker's pushes to a PS arrive in
        # order with none lost or duplicated, and logs (worker, ps, step, t) per update.
        self.check_provenance = check_provenance
        self.provenance: List[Tuple[int, int, int, int]] = []
        self._last_step: Dict[Tuple[int, int], int] = {}
        self._push_step: Dict[int, int] = {}

    # -- PS service thread -------------------------------------------------------------------------
    def _expected_remote(self) -> int:
        W, r = self.env.world, self.env.rank
        n_hosted = sum(1 for p in range(self.plan.num_ps) if self.plan.host_rank(p, W) == r)
        return n_hosted * (W - 1) * self.steps

    def start(self) -> None:
        if self.env.world == 1 or self._expected_remote() == 0:
            return
        self._thread = threading.Thread(target=self._serve, name="ps-service", daemon=True)
        self._thread.start()

    def _serve(self) -> None:
        try:
            dev = self.params.device
            stream = torch.cuda.Stream(device=dev) if self.params.is_cuda else None
            if stream is not None:
                torch.cuda.set_device(dev)
            with _stream_ctx(stream):
                for _ in range(self._expected_remote()):
                    v = self.mailbox.pop(600.0)
                    if v is None:
                        raise TimeoutError("async PS: no arrival within 600 s")
                    w, p = mbox.decode(v)
                    ps = self.servers[p]
                    g = self.pair_groups[(w, self.env.rank)]
                    hdr = None
                    if self.check_provenance:
                        hdr = torch.empty(2, dtype=torch.float64, device=dev)
                        dist.recv(hdr, src=w, group=g)
                    dist.recv(ps.gbuf, src=w, group=g)
                    if hdr is not None:
                        self._verify(w, p, hdr, ps.gbuf)
                    with ps.exclusive():
                        ps.update_own(ps.gbuf, self.grad_scale)
                        if hdr is not None:
                            self.provenance.append((w, p, int(hdr[0].item()), ps.t))
                        dist.send(ps.params, dst=w, group=g)
                    self.served += 1
        except BaseException as e:  # surfaced by join()
            self._error = e

    def _verify(self, w: int, p: int, hdr: torch.Tensor, g: torch.Tensor) -> None:
        step, want = int(hdr[0].item()), float(hdr[1].item())
        got = float(g.double().sum().item())
        if got != want:
            raise RuntimeError(f"provenance: PS {p} received gradient bytes from worker {w} "
                               f"step {step} that differ from what it pushed ({got} != {want})")
        last = self._last_step.get((w, p), -1)
        if step != last + 1:
            raise RuntimeError(f"provenance: PS {p} got worker {w} step {step} after step "
                               f"{last} (lost, duplicated or reordered push)")
        self._last_step[(w, p)] = step

    def verify_provenance(self) -> None:
        """After join(): every hosted PS applied exactly `steps` pushes of every remote
        worker, each once, in step order, and its step counter advanced once per push."""
        for p, ps in self.servers.items():
            for w in range(self.env.world):
                if w == self.env.rank:
                    continue
                steps = [s for (ww, pp, s, _) in self.provenance if ww == w and pp == p]
                if steps != list(range(self.steps)):
                    raise RuntimeError(f"provenance: PS {p} / worker {w} steps {steps[:5]}...")
            ts = [t for (_, pp, _, t) in self.provenance if pp == p]
            if ts != sorted(ts) or len(set(ts)) != len(ts):
                raise RuntimeError(f"provenance: PS {p} step counter not strictly increasing")

    @contextlib.contextmanager
    def paused(self):
        """Checkpoint hook: the service thread updates a PS only under its lock (on its
        stream), so holding every hosted PS's lock with its stream drained is a consistent
        snapshot of parameters, m, v and t."""
        with contextlib.ExitStack() as held:
            for ps in self.servers.values():
                held.enter_context(ps.lock)
                if ps._stream is not None:
                    ps.stream.synchronize()
            yield

    def join(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            raise RuntimeError("async PS service failed") from self._error

    # -- worker side ----------------------------------------------------------------------------------
    def push_pull(self) -> None:
        W, r = self.env.world, self.env.rank
        for p in range(self.plan.num_ps):
            host = self.plan.host_rank(p, W)
            (lo, hi), = self.plan.ps_segments(p)
            if host == r:
                ps = self.servers[p]
                with ps.exclusive():
                    ps.update_own(self.grads[lo:hi], self.grad_scale)
                    self.params[lo:hi].copy_(ps.params)
            else:
                g = self.pair_groups[(r, host)]
                self.remote_boxes[host].push(mbox.encode(r, p))
                if self.check_provenance:
                    step = self._push_step.get(p, 0)
                    self._push_step[p] = step + 1
                    hdr = torch.tensor([float(step), float(self.grads[lo:hi].double().sum())],
                                       dtype=torch.float64, device=self.grads.device)
                    dist.send(hdr, dst=host, group=g)
                dist.send(self.grads[lo:hi], dst=host, group=g)
                dist.recv(self.params[lo:hi], src=host, group=g)

    def close(self) -> None:
        if self.mailbox is not None:
            self.mailbox.close()
