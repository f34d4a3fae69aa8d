#!/usr/bin/env python3
"""A/B of the sync runner's comm-stream hand-off on the one-GPU W > 1 rehearsal
(--force-collectives --exchange $EXCHANGE, xgmi or rccl): event record / wait (mode 0), READY
flag + gate for every segment but the first (1), for every segment (2, default).
Alternating timed windows on one box; prints ms/step per window and the medians."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.config import TrainConfig  # noqa: E402
from ddl_amd.parallel.comm import DistEnv  # noqa: E402
from ddl_amd.parallel.roles import Trainer  # noqa: E402
from ddl_amd.utils.data import synthetic_mnist  # noqa: E402

STEPS = int(os.environ.get("STEPS", "200"))
EXCHANGE = os.environ.get("EXCHANGE", "xgmi")  # xgmi | rccl
data = synthetic_mnist()


def mk(flags):
    tr = Trainer(TrainConfig(mode="sync", shard="flat", steps=10000, eval_every=0, engine="hip",
                             quiet=True, data_sharding="stride", force_collectives=True,
                             exchange_backend=EXCHANGE),
                 DistEnv(0, 1, 0, torch.device("cuda", 0)), dataset=data)
    tr.exchange.runner.set_ready_flags(flags)
    return tr


MODES = (0, 1, 2)
trs = {m: mk(m) for m in MODES}
res = {m: [] for m in MODES}
step = {m: 0 for m in MODES}
for f, tr in trs.items():  # warm both
    for _ in range(100):
        tr.train_step(step[f]); step[f] += 1
torch.cuda.synchronize()
for rep in range(4):
    for f in MODES:
        tr = trs[f]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(STEPS):
            tr.train_step(step[f]); step[f] += 1
        torch.cuda.synchronize()
        res[f].append(1e3 * (time.perf_counter() - t0) / STEPS)
        print(f"rep {rep} ready_flags={f}: {res[f][-1]:.4f} ms/step", flush=True)
for f in MODES:
    print(f"median ready_flags={f}: {statistics.median(res[f]):.4f} ms/step")
