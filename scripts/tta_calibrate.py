#!/usr/bin/env python3
"""Calibrate the hard synthetic set (utils/data.py synthetic_mnist_hard): one reference epoch
(500 steps of batch 100, Adam 1e-4, keep 0.5, eval every 10 steps) per difficulty setting on
one GPU, final test accuracy and time to 95 %.

    python3 scripts/tta_calibrate.py 'styles=4,noise=0.55,mix=0.35,shift=4,contrast=0.35' ...
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import HARD, synthetic_mnist, synthetic_mnist_hard
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    settings = sys.argv[1:] or [",".join(f"{k}={v}" for k, v in HARD.items())]
    for spec in ["easy"] + settings:
        t0 = time.time()
        if spec == "easy":
            data = synthetic_mnist()
        else:
            kw = {}
            for kv in spec.split(","):
                k, v = kv.split("=")
                kw[k] = int(v) if k in ("styles", "shift") else float(v)
            data = synthetic_mnist_hard(**kw)
        gen = time.time() - t0
        cfg = TrainConfig(mode="single", shard="none", steps=500, batch_size=100, eval_every=10,
                          engine="hip" if dev.type == "cuda" else "torch", quiet=True,
                          target_acc=0.95)
        tr = Trainer(cfg, DistEnv(device=dev), dataset=data)
        s = tr.train()
        accs = [round(h["acc"], 4) for h in tr.history]
        print(f"{spec:60s} final {s['final_acc']:.4f}  t95 {s['time_to_target']}  "
              f"acc@100/200/300/400 {accs[10] if len(accs) > 10 else None} "
              f"{accs[20] if len(accs) > 20 else None} {accs[30] if len(accs) > 30 else None} "
              f"{accs[40] if len(accs) > 40 else None}  (gen {gen:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
