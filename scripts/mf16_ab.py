#!/usr/bin/env python3
"""A/B of CFG_MF16 (16x16x4 MFMA + LDS-DMA one-wave tiles, gemm.h mainloop_dma16) on the real
training step (native runner, W = 1), interleaved rounds in one process.

Variants: the engine defaults; the conv backward ops (data + weight gradients of conv4..conv2)
on config 14 with their default splits and with the splits scaled by --scales; the same plus
the conv2-4 forwards; data-gradient-only and weight-gradient-only.

usage: python scripts/mf16_ab.py [--steps 300] [--rounds 3] [--scales 1,2]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FWD = (1, 2, 3)
DGRAD = (10, 12, 14)
WGRAD = (11, 13, 15)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--scales", default="1,2")
    ap.add_argument("--only", default="", help="';'-separated variant names")
    ap.add_argument("--profile", default="",
                    help="run only this variant for --steps steps (under rocprofv3)")
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
    base = {"cfg": e.get_cfg(), "splits": e.get_splits(), "workers": e.get_workers(),
            "wide": e.get_wide()}

    def variant(ops, scale=1.0):
        s = {k: list(v) for k, v in base.items()}
        for op in ops:
            s["cfg"][op] = 14
            s["splits"][op] = max(1, int(round(s["splits"][op] * scale)))
        return s

    scheds = {"default": base}
    for sc in [float(v) for v in a.scales.split(",")]:
        scheds[f"bwd14 x{sc:g}"] = variant(DGRAD + WGRAD, sc)
        scheds[f"all14 x{sc:g}"] = variant(FWD + DGRAD + WGRAD, sc)
    scheds["dgrad14"] = variant(DGRAD)
    scheds["wgrad14"] = variant(WGRAD)
    if a.only:
        keep = set(a.only.split(";"))
        scheds = {k: v for k, v in scheds.items() if k in keep or k == "default"}
    if a.profile:
        scheds = {a.profile: scheds[a.profile]}
        a.rounds = 1
    res = {k: [] for k in scheds}
    step = 0
    for r in range(a.rounds):
        for name, s in scheds.items():
            e.set_cfg(s["cfg"])
            e.set_splits(s["splits"])
            e.set_workers(s["workers"])
            e.set_wide(s["wide"])
            for _ in range(30):
                tr.train_step(step)
                step += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.train_step(step)
                step += 1
            torch.cuda.synchronize()
            res[name].append(1e6 * (time.perf_counter() - t0) / a.steps)
        print(f"round {r} done", flush=True)
    for name, ts in res.items():
        print(f"{name:16s} us/step min {min(ts):7.1f}  all {' '.join(f'{t:.1f}' for t in ts)}",
              flush=True)


if __name__ == "__main__":
    main()
