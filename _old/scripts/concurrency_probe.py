#!/usr/bin/env python3
"""Step time of the native runner for engine concurrency (two streams) x local-update
placement (main stream vs comm stream).  VARIANTS="c1l1,c0l1,..." (c = concurrent wgrad
stream, l = local updates on the main stream), STEPS=200."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.config import TrainConfig  # noqa: E402
from ddl_amd.parallel.comm import DistEnv  # noqa: E402
from ddl_amd.parallel.roles import Trainer  # noqa: E402
from ddl_amd.utils.data import synthetic_mnist  # noqa: E402


def main():
    data = synthetic_mnist(n_train=20000, n_test=1000)
    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    n = int(os.environ.get("STEPS", "200"))
    variants = os.environ.get("VARIANTS", "c0l1d1,c0l1d0,c1l1d0,c0l0d1,c0l1d1,c0l1d0").split(",")
    cfg = TrainConfig(mode="sync", shard="contiguous", steps=400, batch_size=100,
                      eval_every=0, engine="hip", quiet=True)
    tr = Trainer(cfg, env, dataset=data)
    for v in variants:
        conc, local = v[1] == "1", v[3] == "1"
        dual = len(v) < 6 or v[5] == "1"
        tr.engine.set_concurrent(conc)
        tr.engine.set_dual(dual)
        tr.exchange.runner.set_local_on_main(local)
        for i in range(20):
            tr.train_step(i)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(20, 20 + n):
            tr.train_step(i)
        torch.cuda.synchronize()
        print(f"{v}: concurrent={conc} local_on_main={local} dual={dual}: "
              f"{1e6 * (time.perf_counter() - t) / n:.1f} us/step", flush=True)


if __name__ == "__main__":
    main()
