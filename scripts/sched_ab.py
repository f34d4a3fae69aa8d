#!/usr/bin/env python3
"""A/B of per-op GEMM schedules on the real training step (native runner, W = 1): the
engine defaults vs schedules from step_tune.py --json files, interleaved rounds, one process.

usage: python scripts/sched_ab.py tuned1.json [tuned2.json ...] [--steps 300] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tuned", nargs="*")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--splits-variants", default="",
                    help="';'-separated split overrides of the defaults, each 'op=s,op=s'")
    ap.add_argument("--cfg-variants", default="",
                    help="';'-separated tile-config overrides 'op=cfg[:split],...' (name=... first "
                         "to label it)")
    ap.add_argument("--wide-variants", default="",
                    help="';'-separated split-K reduce overrides 'op=inl|wide,...' (inl: the "
                         "in-launch last arriver; wide: the separate reduce kernel); a "
                         "'name=...' first labels it, 'op=cfg:split' items set the config and "
                         "'bf=mask' the dual_bfirst mask")
    ap.add_argument("--bfirst-variants", default="",
                    help="';'-separated dual_bfirst masks (bit op: that dual dispatches its "
                         "second problem first)")
    ap.add_argument("--tail-variants", default="",
                    help="';'-separated optimizer-tail layouts 'first:f4' (first: tail blocks "
                         "ahead of the GEMM blocks; f4: float4 per tail block, default 0:1024)")
    a = ap.parse_args()
    import torch
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import synthetic_mnist

    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", shard="flat", steps=10 ** 6, batch_size=100, eval_every=0,
                      engine="hip", quiet=True, data_sharding="stride")
    tr = Trainer(cfg, env, dataset=synthetic_mnist())
    e = tr.engine.eng
    scheds = {"default": {"cfg": e.get_cfg(), "splits": e.get_splits(), "wide": e.get_wide(),
                          "bfirst": e.get_dual_bfirst()}}
    for p in a.tuned:
        scheds[os.path.basename(p)] = json.load(open(p))
    for v in filter(None, a.splits_variants.split(";")):
        sp = list(scheds["default"]["splits"])
        for kv in v.split(","):
            op, val = kv.split("=")
            sp[int(op)] = int(val)
        scheds["splits[" + v + "]"] = dict(scheds["default"], splits=sp)
    for v in filter(None, a.cfg_variants.split(";")):
        cf = list(scheds["default"]["cfg"])
        sp = list(scheds["default"]["splits"])
        label = v
        for kv in v.split(","):
            if kv.startswith("name="):
                label = kv[5:]
                continue
            op, val = kv.split("=")
            c, _, spl = val.partition(":")
            cf[int(op)] = int(c)
            if spl:
                sp[int(op)] = int(spl)
        scheds["cfg[" + label + "]"] = dict(scheds["default"], cfg=cf, splits=sp)
    for v in filter(None, a.wide_variants.split(";")):
        wd = list(scheds["default"]["wide"])
        cf = list(scheds["default"]["cfg"])
        sp = list(scheds["default"]["splits"])
        label = v
        bf = scheds["default"]["bfirst"]
        for kv in v.split(","):
            if kv.startswith("name="):
                label = kv[5:]
                continue
            op, val = kv.split("=")
            if op == "bf":
                bf = int(val)
                continue
            if val in ("inl", "wide"):
                wd[int(op)] = (1 << 20) if val == "inl" else 1
            else:
                c, _, spl = val.partition(":")
                cf[int(op)] = int(c)
                if spl:
                    sp[int(op)] = int(spl)
        scheds["wide[" + label + "]"] = dict(scheds["default"], wide=wd, cfg=cf, splits=sp, bfirst=bf)
    for v in filter(None, a.tail_variants.split(";")):
        fi, f4 = v.split(":")
        scheds["tail[" + v + "]"] = dict(scheds["default"], tail=(int(fi), int(f4)))
    for v in filter(None, a.bfirst_variants.split(";")):
        scheds["bfirst[" + v + "]"] = dict(scheds["default"], bfirst=int(v))
    res = {k: [] for k in scheds}
    step = 0
    for _ in range(a.rounds):
        for name, s in scheds.items():
            e.set_cfg(s["cfg"])
            e.set_splits(s["splits"])
            e.set_wide(s["wide"])
            e.set_dual_bfirst(s["bfirst"])
            tr.exchange.runner.set_tail_cfg(*s.get("tail", (0, 1024)))
            for _ in range(20):
                tr.train_step(step)
                step += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.train_step(step)
                step += 1
            torch.cuda.synchronize()
            res[name].append(1e6 * (time.perf_counter() - t0) / a.steps)
    for name, ts in res.items():
        print(f"{name:48s} us/step min {min(ts):7.1f}  all {' '.join(f'{t:.1f}' for t in ts)}")


if __name__ == "__main__":
    main()
