#!/usr/bin/env python3
"""Run N default native-runner training steps (for rocprofv3 --pmc collection).

    python3 scripts/pmc_probe.py [SCHED_JSON] [STEPS]
SCHED_JSON: a runner_tune.py / sched JSON (cfg, splits, wide) to run instead of the
defaults; STEPS: training steps (default 20)."""
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
if len(sys.argv) > 1 and sys.argv[1].endswith(".json"):
    import json
    sc = json.load(open(sys.argv[1]))
    e = tr.engine.eng
    e.set_cfg(sc["cfg"])
    e.set_splits(sc["splits"])
    e.set_wide(sc["wide"])
for i in range(int(sys.argv[-1]) if sys.argv[-1].isdigit() else 20):
    tr.train_step(i)
torch.cuda.synchronize()
print("done")
