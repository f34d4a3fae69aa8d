#!/usr/bin/env python3
"""Stress the xGMI exchange protocol with W processes on one GPU: every iteration each rank
fills its gradients with a pattern that depends on (rank, iteration), runs one exchange of every
bucket with the self-test update (w := sum over ranks of g) and checks the result exactly.
Optionally runs real training steps in between (--train-every k) so the comm-stream kernels
overlap the backward GEMMs like in the real step.

usage: python scripts/xgmi_stress.py [--world 4] [--iters 200] [--train-every 0]
"""
import argparse
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, world, port, iters, train_every, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DDL_DIST_BACKEND="gloo",
                      DDL_XGMI_TIMEOUT_S="20")
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed()
        cfg = TrainConfig(mode="sync", shard="flat", steps=10 ** 6, batch_size=100, eval_every=0,
                          engine="hip", quiet=True, data_sharding="stride",
                          exchange_backend="xgmi")
        tr = Trainer(cfg, env, dataset=synthetic_mnist(2000, 500, seed=5))
        ex = tr.exchange
        assert ex.peer is not None
        n = tr.params.numel()
        idx = torch.arange(n, device=tr.params.device)
        bad = 0
        first = None
        step = 0
        import time
        t0 = time.time()
        for it in range(iters):
            if rank == 0 and it % 10 == 0:
                print(f"iter {it} {time.time() - t0:.1f}s", flush=True)
            if train_every and it % train_every == 0:
                tr.train_step(step)
                step += 1
            # exact in fp32: small integers
            pat = ((idx * 7 + it * 13) % 31 + 1).to(torch.float32)
            tr.grads.copy_(pat * float(rank + 1))
            torch.cuda.synchronize()
            ex.runner.peer_selftest_step()
            want = pat * float(world * (world + 1) // 2)
            for lo, hi in tr.plan.bucket_ranges:
                d = (tr.params[lo:hi] != want[lo:hi])
                if bool(d.any()):
                    bad += 1
                    if first is None:
                        k = int(d.nonzero()[0]) + lo
                        first = (it, k, float(tr.params[k]), float(want[k]))
                    break
        err = ex.peer.error()
        with open(os.path.join(out, f"stress{rank}.txt"), "w") as f:
            f.write(f"{bad} {first} {err}\n")
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


def main():
    ap = argparse.ArgumentParser()
    # at most 4 ranks on one card: 8 oversubscribe the hardware queues (see tests/test_xgmi_gpu.py)
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--train-every", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/stress")
    a = ap.parse_args()
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.makedirs(a.out, exist_ok=True)
    mp.spawn(rank_main, args=(a.world, port, a.iters, a.train_every, a.out), nprocs=a.world,
             join=True)
    tot = 0
    for r in range(a.world):
        line = open(os.path.join(a.out, f"stress{r}.txt")).read().strip()
        print(f"rank {r}: mismatching iterations / first (iter, index, got, want) / err: {line}")
        tot += int(line.split()[0])
    print("TOTAL_BAD", tot, flush=True)


if __name__ == "__main__":
    main()
