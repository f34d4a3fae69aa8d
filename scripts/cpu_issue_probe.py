#!/usr/bin/env python3
"""Is the step CPU-issue-bound?  Times N train_step() calls without any synchronisation (host
issue time, as long as the queue does not fill) against the same N steps to GPU completion,
for the default W = 1 step and the forced W > 1 rehearsals (--force-collectives, RCCL / xGMI)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.config import TrainConfig  # noqa: E402
from ddl_amd.parallel.comm import init_distributed  # noqa: E402
from ddl_amd.parallel.roles import Trainer  # noqa: E402
from ddl_amd.utils.data import synthetic_mnist  # noqa: E402


def main():
    env = init_distributed()
    data = synthetic_mnist()
    n = 60
    for name, force, ex in (("local", False, "auto"), ("forced-rccl", True, "rccl"),
                            ("forced-xgmi", True, "xgmi")):
        cfg = TrainConfig(mode="sync", shard="flat", steps=400, batch_size=100, eval_every=0,
                          engine="hip", quiet=True, data_sharding="stride",
                          force_collectives=force, exchange_backend=ex)
        tr = Trainer(cfg, env, dataset=data)
        for i in range(30):
            tr.train_step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(30, 30 + n):
            tr.train_step(i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:12s} host issue {1e6 * (t1 - t0) / n:7.1f} us/step   "
              f"to completion {1e6 * (t2 - t0) / n:7.1f} us/step", flush=True)


if __name__ == "__main__":
    main()
