"""Checkpoint / resume with the reference's variable naming.

The reference never checkpoints; its only stable layout is the variable naming:
worker variables ``mnist/v0..v13`` (``mnist_sync/model/model.py:17,24-86``), PS variables
``ParameterServer/v{i}`` (``mnist_sync_sharding/parameter_server.py:56-60``) with TF1 Adam
slots ``/Adam`` (m), ``/Adam_1`` (v) and per-PS ``beta1_power``/``beta2_power``
[TF-semantics].

Layout of a checkpoint directory (safetensors, no pickle):

  manifest.json                 plan, world, step, per-PS step counters
  worker{r}.safetensors         mnist/v{i} for worker r (sync: only worker 0)
  ps{p}.safetensors             ParameterServer/v{i}[@a:b], .../Adam, .../Adam_1,
                                ParameterServer/beta1_power, beta2_power

A PS that owns only part of a tensor (``flat`` plans) stores the piece ``@a:b`` (element
range inside the tensor).  Resume stitches pieces back into whole tensors and re-shards
them under the *current* plan, so a job can resume with a different PS count or policy.
"""
from __future__ import annotations

import json
import os
import sys
from typing import Dict, List, Tuple

import torch
from safetensors.torch import save_file, load_file

from ..models.layout import TENSORS


def _pieces(plan, lo: int, hi: int) -> List[Tuple[int, int, int, int]]:
    """(tensor id, a, b, plan offset) pieces of plan range [lo, hi)."""
    out = []
    for t in TENSORS:
        o = plan.tensor_offsets[t.index]
        a, b = max(lo, o), min(hi, o + t.numel)
        if a < b:
            out.append((t.index, a - o, b - o, a))
    return out


def _name(i: int, a: int, b: int, n: int) -> str:
    return f"ParameterServer/v{i}" if (a == 0 and b == n) else f"ParameterServer/v{i}@{a}:{b}"


def save(trainer, path: str) -> None:
    import contextlib
    import torch.distributed as dist
    os.makedirs(path, exist_ok=True)
    env, plan = trainer.env, trainer.plan
    asyncm = trainer.cfg.mode == "async"
    ex = trainer.exchange
    drain = getattr(ex, "drain_round", None)  # async native step: this worker's round is back
    if drain is not None:
        drain()
    if trainer.params.is_cuda:
        # every queued step (and its exchange kernels) must have finished, and must not have
        # failed: a checkpoint of parameters a timed-out exchange left half-updated is refused
        torch.cuda.synchronize(trainer.params.device)
    if getattr(ex, "native", False) and hasattr(ex, "check"):
        ex.check()
    sync_state = getattr(ex, "sync_ps_state", None)  # replicated optimizer state -> the PS
    if sync_state is not None:
        sync_state()
    # async: the PS service keeps applying other workers' pushes.  Snapshot the hosted PS
    # state (parameters, m, v and the step counter t) with the service paused, so it is one
    # consistent PS step; the pause ends before any collective below (a peer may be waiting
    # for this PS to serve its push before it reaches its own checkpoint).
    pause = getattr(ex, "paused", None)
    with (pause() if pause is not None else contextlib.nullcontext()):
        snaps = {p: _ps_snapshot(trainer, plan, ps) for p, ps in trainer.servers.items()}
    if asyncm or env.rank == 0:
        w = {}
        for t in TENSORS:
            o = plan.tensor_offsets[t.index]
            w[f"mnist/v{t.index}"] = trainer.params[o:o + t.numel].detach().view(t.shape).cpu().contiguous()
        save_file(w, os.path.join(path, f"worker{env.rank}.safetensors"))
    for p, (d, _) in snaps.items():
        save_file(d, os.path.join(path, f"ps{p}.safetensors"))
    # every PS's own step counter (PSes are hosted by different ranks), over the host-only
    # control group: in async mode a peer may still need this rank's PS service (an RCCL
    # session or an xGMI apply) to finish its round before it reaches its own save, and an RCCL
    # collective here could queue on a hardware queue in front of that serve kernel
    local_t = {p: t for p, (_, t) in snaps.items()}
    all_t = [local_t]
    grp = getattr(env, "ctrl", None)
    if env.world > 1:
        all_t = [None] * env.world
        dist.all_gather_object(all_t, local_t, group=grp)
    if env.rank == 0:
        ps_t = {}
        for d in all_t:
            ps_t.update({str(k): v for k, v in d.items()})
        # the PS ranges themselves: two plans with one policy and PS count can
        # still differ (flat vs segment-aligned flat), and a PS step counter is only valid on
        # the ranges it counted
        man = dict(policy=plan.policy, num_ps=plan.num_ps, world=env.world, mode=trainer.cfg.mode,
                   global_step=trainer.global_step, ps_t=ps_t,
                   ps_segments=[[list(map(int, r)) for r in plan.ps_segments(p)]
                                for p in range(plan.num_ps)])
        with open(os.path.join(path, "manifest.json"), "w") as f:
            json.dump(man, f, indent=1)
    if env.world > 1:
        dist.barrier(group=grp)


def _ps_snapshot(trainer, plan, ps) -> Tuple[Dict[str, torch.Tensor], int]:
    """Host copies of one PS's tensors under the reference's names, and its step counter."""
    d: Dict[str, torch.Tensor] = {}
    for (lo, hi), off in zip(ps.segments, ps.seg_off):
        for i, a, b, po in _pieces(plan, lo, hi):
            n = TENSORS[i].numel
            base = _name(i, a, b, n)
            s0 = off + (po - lo)
            src = ps.params[s0:s0 + (b - a)] if ps.params is not None else trainer.params[po:po + (b - a)]
            d[base] = src.detach().cpu().contiguous()
            d[base + "/Adam"] = ps.m[s0:s0 + (b - a)].detach().cpu().contiguous()
            if ps.v is not None:
                d[base + "/Adam_1"] = ps.v[s0:s0 + (b - a)].detach().cpu().contiguous()
    b1, b2 = ps.h.beta1 ** ps.t, ps.h.beta2 ** ps.t
    d["ParameterServer/beta1_power"] = torch.tensor([b1], dtype=torch.float32)
    d["ParameterServer/beta2_power"] = torch.tensor([b2], dtype=torch.float32)
    return d, ps.t


def _stitch(path: str, num_ps: int) -> Tuple[Dict[int, Dict[str, torch.Tensor]], List[float]]:
    full: Dict[int, Dict[str, torch.Tensor]] = {}
    powers = []
    for p in range(num_ps):
        fn = os.path.join(path, f"ps{p}.safetensors")
        d = load_file(fn)
        powers.append(float(d.pop("ParameterServer/beta1_power")[0]))
        d.pop("ParameterServer/beta2_power", None)
        for k, v in d.items():
            if k.endswith("/Adam"):
                base, slot = k[:-len("/Adam")], "m"
            elif k.endswith("/Adam_1"):
                base, slot = k[:-len("/Adam_1")], "v"
            else:
                base, slot = k, "w"
            name = base.split("/")[1]
            i = int(name.split("@")[0][1:])
            a, b = 0, TENSORS[i].numel
            if "@" in name:
                a, b = map(int, name.split("@")[1].split(":"))
            ent = full.setdefault(i, {})
            if slot not in ent:
                ent[slot] = torch.zeros(TENSORS[i].numel, dtype=torch.float32)
            ent[slot][a:b] = v
    return full, powers


def load(trainer, path: str) -> None:
    with open(os.path.join(path, "manifest.json")) as f:
        man = json.load(f)
    env, plan = trainer.env, trainer.plan
    wf = os.path.join(path, f"worker{env.rank}.safetensors")
    if not os.path.exists(wf):
        wf = os.path.join(path, "worker0.safetensors")
    w = load_file(wf)
    for t in TENSORS:
        o = plan.tensor_offsets[t.index]
        trainer.params[o:o + t.numel].copy_(w[f"mnist/v{t.index}"].reshape(-1))
    full, _ = _stitch(path, man["num_ps"])
    ts = [v for v in man["ps_t"].values() if v is not None]
    t_resume = max(ts) if ts else 0
    for p, ps in trainer.servers.items():
        for (lo, hi), off in zip(ps.segments, ps.seg_off):
            for i, a, b, po in _pieces(plan, lo, hi):
                s0 = off + (po - lo)
                ps.m[s0:s0 + (b - a)].copy_(full[i]["m"][a:b])
                if ps.v is not None and "v" in full[i]:
                    ps.v[s0:s0 + (b - a)].copy_(full[i]["v"][a:b])
                if ps.params is not None:
                    ps.params[s0:s0 + (b - a)].copy_(full[i]["w"][a:b])
        same_plan = man["policy"] == plan.policy and man["num_ps"] == plan.num_ps
        if "ps_segments" in man:
            same_plan = same_plan and man["ps_segments"] == [
                [list(map(int, r)) for r in plan.ps_segments(q)] for q in range(plan.num_ps)]
        elif same_plan and p == next(iter(trainer.servers)):
            # a manifest from before round 5 carries no PS ranges: policy + PS count is the best
            # identity it offers, so the per-PS counters are kept on that basis (said once)
            print("[ddl_amd] checkpoint manifest has no ps_segments: per-PS step counters "
                  "restored by policy and PS count only", file=sys.stderr)
        ps.t = int(man["ps_t"].get(str(p)) or t_resume) if same_plan else t_resume
    trainer.global_step = int(man["global_step"])
    load_state = getattr(trainer.exchange, "load_ps_state", None)
    if load_state is not None:  # PS chunks -> the exchange's replicated optimizer state
        load_state()
