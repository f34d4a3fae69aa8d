#!/usr/bin/env python3
"""Step time of the W = 1 native runner with the optimizer tail (csrc/kernels/tail.h) off and
in several placements / block sizes, interleaved rounds in one process.

usage: python scripts/tail_probe.py [--steps 300] [--rounds 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shard", default="flat")
    a = ap.parse_args()
    import torch
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import synthetic_mnist

    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", shard=a.shard, steps=10 ** 6, batch_size=100, eval_every=0,
                      engine="hip", quiet=True, data_sharding="stride")
    tr = Trainer(cfg, env, dataset=synthetic_mnist())
    run = tr.exchange.runner
    variants = [("off", None)] + [(f"{'first' if f else 'last'}-f4x{n}", (f, n))
                                  for f in (1, 0) for n in (512, 1024, 2048, 4096)]
    res = {k: [] for k, _ in variants}
    step = 0
    for _ in range(a.rounds):
        for name, v in variants:
            if v is None:
                run.set_use_tail(False)
            else:
                run.set_use_tail(True)
                run.set_tail_cfg(*v)
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
        print(f"{name:16s} us/step min {min(ts):7.1f}  all {' '.join(f'{t:.1f}' for t in ts)}")


if __name__ == "__main__":
    main()
