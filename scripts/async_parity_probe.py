#!/usr/bin/env python3
"""W = 1 parity probe: async over xGMI (native runner / Python push_pull) vs the local step.
Prints the per-tensor max |diff| of the parameters after each of the first steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.config import TrainConfig  # noqa: E402
from ddl_amd.parallel.comm import DistEnv  # noqa: E402
from ddl_amd.parallel.roles import Trainer  # noqa: E402
from ddl_amd.utils.data import synthetic_mnist  # noqa: E402

DEV = torch.device("cuda", 0)
data = synthetic_mnist(n_train=3000, n_test=600, seed=11)


def mk(**kw):
    base = dict(mode="async", shard="flat", batch_size=100, eval_every=0, engine="hip",
                quiet=True, steps=12)
    base.update(kw)
    return Trainer(TrainConfig(**base), DistEnv(0, 1, 0, DEV), dataset=data)


def tensors(tr):
    out = []
    for t in range(14):
        lo, hi = tr.plan.tensor_extent(t)
        out.append(tr.params[lo:hi].clone())
    return out


steps = int(os.environ.get("STEPS", "3"))
runs = {"local": mk(), "xgmi_native": mk(exchange_backend="xgmi")}
os.environ["DDL_ASYNC_NATIVE"] = "0"
runs["xgmi_python"] = mk(exchange_backend="xgmi")
for name, tr in runs.items():
    if not tr.async_as_sync:
        tr.exchange.steps = steps
        tr.exchange.start()
ref0 = tensors(runs["local"])
for name, tr in runs.items():
    d = max(float((a - b).abs().max()) for a, b in zip(tensors(tr), ref0))
    print(f"init {name}: max diff {d:.3g}")
for i in range(steps):
    for name, tr in runs.items():
        tr.train_step(i)
    for name, tr in runs.items():
        if not tr.async_as_sync:
            tr.exchange.drain_round() if tr.exchange.runner is not None else None
    torch.cuda.synchronize()
    ref = tensors(runs["local"])
    for name, tr in runs.items():
        if name == "local":
            continue
        diffs = [float((a - b).abs().max()) for a, b in zip(tensors(tr), ref)]
        print(f"step {i} {name}: " + " ".join(f"{d:.2g}" for d in diffs))
for name, tr in runs.items():
    if not tr.async_as_sync:
        tr.exchange.join()
print("done")
