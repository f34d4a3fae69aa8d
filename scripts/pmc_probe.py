#!/usr/bin/env python3
"""Run N default native-runner training steps (for rocprofv3 --pmc collection)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.config import TrainConfig  # noqa: E402
from ddl_amd.parallel.comm import DistEnv  # noqa: E402
from ddl_amd.parallel.roles import Trainer  # noqa: E402
from ddl_amd.utils.data import synthetic_mnist  # noqa: E402

data = synthetic_mnist(n_train=5000, n_test=500)
tr = Trainer(TrainConfig(mode="sync", shard="contiguous", steps=50, eval_every=0, engine="hip",
                         quiet=True), DistEnv(0, 1, 0, torch.device("cuda", 0)), dataset=data)
if os.environ.get("DDL_PROBE_MF16") == "1":  # conv backward on CFG_MF16 (splits x2)
    e = tr.engine.eng
    cfg, spl = e.get_cfg(), e.get_splits()
    for op in (10, 11, 12, 13, 14, 15):
        cfg[op], spl[op] = 14, spl[op] * 2
    e.set_cfg(cfg)
    e.set_splits(spl)
if os.environ.get("DDL_PROBE_SCHED"):  # a runner_tune.py / sched JSON (cfg, splits, ...)
    import json
    sc = json.load(open(os.environ["DDL_PROBE_SCHED"]))
    e = tr.engine.eng
    e.set_cfg(sc["cfg"])
    e.set_splits(sc["splits"])
    e.set_workers(sc["workers"])
    e.set_wide(sc["wide"])
for i in range(int(os.environ.get("STEPS", "20"))):
    tr.train_step(i)
torch.cuda.synchronize()
print("done")
