#!/usr/bin/env python3
"""Where the driver window's fixed cost goes (bench.py --steps 20 --warmup 5 reads ~3 us/step
above a 300-step window).  W = 1, the bench's trainer: after the prewarm, windows of K steps
bracketed like bench.py (synchronize, perf_counter, K train_step calls, synchronize) with
host-side stamps after every train_step call and GPU events at both ends.

usage: python scripts/window_probe.py [--k 20] [--windows 8] [--prewarm 1000]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--prewarm", type=int, default=1000)
    ap.add_argument("--gc-off", action="store_true", help="gc.disable() around the windows "
                    "(as bench.py's timed_run)")
    ap.add_argument("--sched", default="", help="schedule overrides 'op=cfg:split,...'")
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
    if a.sched:
        e = tr.engine.eng
        cf, sp = e.get_cfg(), e.get_splits()
        for kv in a.sched.split(","):
            op, val = kv.split("=")
            c, _, s_ = val.partition(":")
            cf[int(op)] = int(c)
            if s_:
                sp[int(op)] = int(s_)
        e.set_cfg(cf)
        e.set_splits(sp)
        print(f"schedule: cfg {cf} splits {sp}")
    step = 0
    for _ in range(a.prewarm):
        tr.train_step(step)
        step += 1
    torch.cuda.synchronize()
    # steady state: a long window
    t0 = time.perf_counter()
    for _ in range(300):
        tr.train_step(step)
        step += 1
    torch.cuda.synchronize()
    steady = 1e6 * (time.perf_counter() - t0) / 300
    print(f"steady 300-step window: {steady:.1f} us/step")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if a.gc_off:
        import gc
        gc.collect()
        gc.disable()
    for w in range(a.windows):
        for _ in range(5):  # the driver's warmup
            tr.train_step(step)
            step += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        host = []
        for _ in range(a.k):
            tr.train_step(step)
            step += 1
            host.append(time.perf_counter())
        e1.record()
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        gpu = 1e3 * e0.elapsed_time(e1)
        wall = 1e6 * (t1 - t0)
        first = 1e6 * (host[0] - t0)
        per = [1e6 * (host[i] - host[i - 1]) for i in range(1, len(host))]
        print(f"window {w}: wall {wall:7.1f} us = {wall / a.k:6.1f}/step  gpu(events) {gpu:7.1f}"
              f"  wall-gpu {wall - gpu:5.1f}  over steady {wall - a.k * steady:6.1f}  "
              f"host: first call {first:5.1f}, then {min(per):5.1f}-{max(per):5.1f} us/call, "
              f"enqueue done at {1e6 * (t_enq - t0):7.1f}, sync return +{1e6 * (t1 - t_enq):6.1f}")


if __name__ == "__main__":
    main()
