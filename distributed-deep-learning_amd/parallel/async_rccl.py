"""Asynchronous parameter server over point-to-point RCCL, issued natively
(``csrc/kernels/rccl_async.hip``).

Reference (``mnist_async_sharding/worker.py:30-37,88-94``,
``parameter_server.py:94-111``): each worker Sends its gradient shards and blocks in Recv for
the parameters; each PS serves whichever push arrives (``ANY_SOURCE``), applies Adam with its
own step counter and Sends the parameters back.

Here every p2p transfer is part of an exclusive session between two processes (the kernel
file has the deadlock argument): one RCCL communicator, one comm stream and one native comm
thread per process; the initiating worker holds both processes' session locks (POSIX shm) and
posts ``(worker, ps)`` into the host's session mailbox.  This is the RCCL data plane of the
async modes; the xGMI one (``async_xgmi.py``) needs no p2p kernels and is the default on GPUs.
``self_sessions`` (W = 1) runs the exchange as send/recv to itself: the p2p path on one GPU.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Tuple

import torch
import torch.distributed as dist

from ..ops import native
from .comm import DistEnv
from .ps import ParameterServer
from .sharding import ShardPlan


class RcclAsyncUnavailable(RuntimeError):
    pass


class RcclAsyncExchange:
    backend = "rccl"

    def __init__(self, plan: ShardPlan, env: DistEnv, params: torch.Tensor, grads: torch.Tensor,
                 servers: Dict[int, ParameterServer], steps_per_worker: int, job_id: str,
                 optimizer: str = "adam", check_provenance: bool = False):
        if not params.is_cuda or not native.available():
            raise RcclAsyncUnavailable("needs the extension and a GPU")
        if env.world > 1 and env.backend != "nccl":
            raise RcclAsyncUnavailable("needs the nccl (RCCL) default group to exchange the id")
        if optimizer not in ("adam", "momentum", "sgd"):
            raise RcclAsyncUnavailable(f"no '{optimizer}' update")
        P, W, r = plan.num_ps, env.world, env.rank
        for p in range(P):
            if len(plan.ps_segments(p)) != 1:
                raise RcclAsyncUnavailable("async mode needs one contiguous range per PS")
        self.plan, self.env, self.params, self.grads = plan, env, params, grads
        self.servers = servers
        self.steps = steps_per_worker
        self.check_provenance = check_provenance
        self.ranges: List[Tuple[int, int]] = [plan.ps_segments(p)[0] for p in range(P)]
        self.hosts = [plan.host_rank(p, W) for p in range(P)]
        h = next(iter(servers.values())).h if servers else None
        mom = 0.0 if optimizer == "sgd" else (next(iter(servers.values())).momentum
                                              if servers else 0.9)
        hyper = h or _default_hyper()
        ops = native.ops()
        ps_list = [(p, ps.params, ps.m, ps.v, ps.t) for p, ps in servers.items()]
        self.svc = ops.RcclAsync(params, grads, W, r, [tuple(map(int, x)) for x in self.ranges],
                                 [int(x) for x in self.hosts], ps_list,
                                 0 if optimizer == "adam" else 1, hyper.lr, hyper.beta1,
                                 hyper.beta2, hyper.eps, mom, W == 1)
        # communicator: rank 0's unique id over the default group (every rank joins)
        ids = [None]
        if r == 0:
            ids[0] = ops.SyncRunner.unique_id()
        if W > 1:
            dist.broadcast_object_list(ids, src=0)
        self.svc.init_comm(ids[0])
        # session locks (rank 0 creates the segment) and one session mailbox per rank
        if r == 0:
            self.svc.attach_shm(job_id, True)
        if W > 1:
            dist.barrier()
        if r != 0:
            self.svc.attach_shm(job_id, False)
        self.svc.open_boxes(True)
        if W > 1:
            dist.barrier()
        self.svc.open_boxes(False)
        self.served = 0
        self.provenance: List[Tuple[int, int, int, int]] = []

    def _expected(self) -> int:
        W, r = self.env.world, self.env.rank
        return sum(1 for hh in self.hosts if hh == r) * (W - 1) * self.steps

    def start(self) -> None:
        # the PS step counters may have been restored (checkpoint load) after the native object
        # copied them in __init__: hand the current ones over before the service runs
        for p, ps in self.servers.items():
            self.svc.set_t(p, int(ps.t))
        self.svc.start(self._expected(), self.check_provenance)

    def push_pull(self) -> None:
        self.svc.push_pull()

    def _sync_counters(self) -> None:
        for p, ps in self.servers.items():
            n = self.svc.t(p) - ps.t
            ps.t += n
            ps.updates += n

    @contextlib.contextmanager
    def paused(self):
        """Checkpoint hook: no session is served and no update issued inside the block."""
        self.svc.pause()
        try:
            self._sync_counters()
            yield
        finally:
            self.svc.resume()

    def join(self) -> None:
        try:
            self.svc.join()
        finally:
            self._sync_counters()
            self.served = self.svc.served()
            if self.check_provenance:
                # (worker, ps, that worker's round at the PS from 1, PS step) -> rounds from 0
                self.provenance = [(w, p, k - 1, t) for (w, p, k, t) in self.svc.provenance()]

    def verify_provenance(self) -> None:
        """Every hosted PS applied exactly `steps` pushes of every worker, in round order, and
        its step counter advanced once per push."""
        for p in self.servers:
            for w in range(self.env.world):
                steps = [s for (ww, pp, s, _) in self.provenance if ww == w and pp == p]
                if steps != list(range(self.steps)):
                    raise RuntimeError(f"provenance: PS {p} / worker {w} steps {steps[:5]}...")
            ts = [t for (_, pp, _, t) in self.provenance if pp == p]
            if ts != sorted(ts) or len(set(ts)) != len(ts):
                raise RuntimeError(f"provenance: PS {p} step counter not strictly increasing")

    def close(self) -> None:
        pass


def _default_hyper():
    from ..ops.adam import AdamHyper
    return AdamHyper()
