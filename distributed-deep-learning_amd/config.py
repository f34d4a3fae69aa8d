"""One config dataclass + argparse for every entry point.

The reference hard-codes everything: ``epoch = 1``, ``batch_size = 100``
(``mnist_sync/worker.py:41-42``), Adam lr 1e-4 (``mnist_sync/model/model.py:93``),
keep_prob 0.5 (``mnist_sync/worker.py:30``), eval every 10 steps (``:71``), PS/worker
counts from ``sys.argv[2]`` (``-np N``, ``mnist_sync_sharding/parameter_server.py:95``).
Those are the defaults here; ``-np`` is accepted for command-line compatibility.
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass, field, asdict
from typing import Optional

from . import VARIANTS


@dataclass
class TrainConfig:
    mode: str = "sync"              # sync | async | single
    shard: str = "contiguous"       # none | contiguous | greedy | lpt | flat
    num_ps: Optional[int] = None    # default: one PS per worker process (sharded), 1 for 'none'
    epochs: int = 1
    batch_size: int = 100
    steps: Optional[int] = None     # steps per epoch (default total_batch // batch_size = 500)
    lr: float = 1e-4
    optimizer: str = "adam"         # adam | momentum | sgd
    momentum: float = 0.9
    keep_prob: float = 0.5
    eval_every: int = 10            # 0 disables periodic eval
    data: str = "synthetic"
    data_sharding: str = "replicate"  # replicate (reference) | stride
    grad_reduce: str = "sum"        # sum (reference PS sums) | mean
    ref_quirks: bool = False        # reproduce SURVEY.md §2.10 Q1/Q2/Q4
    seed: int = 0
    engine: str = "auto"            # auto | hip | torch
    graph: bool = False             # replay the compute step as HIP graphs (eager is faster)
    overlap: bool = True            # bucketed grad push overlapped with backward
    native_exchange: bool = True    # sync step in the C++ SyncRunner (HIP engine on GPU)
    force_collectives: bool = False  # W = 1: native runner keeps RS/reduce units on a 1-rank comm
    # W > 1 data plane of the native sync runner: rccl (reduce-scatter / all-gather or reduce /
    # broadcast) or xgmi (flat plan: one fused push / owner-Adam / pull kernel per bucket over
    # IPC-mapped peer memory, csrc/kernels/xgmi.hip); auto = rccl
    exchange_backend: str = "auto"
    dist_eval: bool = True          # sync, W > 1: each rank scores 1/W of the test set
    eval_async: bool = False        # HIP engine: periodic eval on a side stream from a snapshot
    check_provenance: bool = False  # async: verify every applied push
    log_jsonl: Optional[str] = None
    checkpoint_dir: Optional[str] = None
    checkpoint_every: int = 0
    resume: bool = False            # continue from checkpoint_dir at its global step
    max_steps: Optional[int] = None  # stop after this many global steps (a preempted run)
    target_acc: Optional[float] = None
    quiet: bool = False
    watchdog_s: float = 600.0

    def to_dict(self):
        return asdict(self)


def add_args(p: argparse.ArgumentParser, mode_default: str = "sync") -> argparse.ArgumentParser:
    d = TrainConfig()
    p.add_argument("-np", dest="np_compat", type=int, default=None,
                   help="reference compatibility: number of PS (parameter_server.py) or "
                        "workers (worker.py)")
    p.add_argument("--variant", choices=sorted(VARIANTS), default=None,
                   help="preset mode/shard named after the reference directories")
    p.add_argument("--mode", default=mode_default, choices=["sync", "async", "single"])
    p.add_argument("--shard", default=d.shard,
                   choices=["none", "contiguous", "greedy", "lpt", "flat"])
    p.add_argument("--num-ps", type=int, default=None)
    p.add_argument("--epochs", type=int, default=d.epochs)
    p.add_argument("--batch-size", type=int, default=d.batch_size)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--lr", type=float, default=d.lr)
    p.add_argument("--optimizer", default=d.optimizer, choices=["adam", "momentum", "sgd"])
    p.add_argument("--keep-prob", type=float, default=d.keep_prob)
    p.add_argument("--eval-every", type=int, default=d.eval_every)
    p.add_argument("--data", default=d.data)
    p.add_argument("--data-sharding", default=d.data_sharding, choices=["replicate", "stride"])
    p.add_argument("--grad-reduce", default=d.grad_reduce, choices=["sum", "mean"])
    p.add_argument("--ref-quirks", action="store_true")
    p.add_argument("--seed", type=int, default=d.seed)
    p.add_argument("--engine", default=d.engine, choices=["auto", "hip", "torch"])
    p.add_argument("--graph", action="store_true", help="replay the engine step as HIP graphs")
    p.add_argument("--no-graph", action="store_true", help="(default)")
    p.add_argument("--check-provenance", action="store_true",
                   help="async: checksum every push and verify order/provenance at the PS")
    p.add_argument("--no-dist-eval", action="store_true",
                   help="every worker scores the full test set (reference behaviour)")
    p.add_argument("--eval-async", action="store_true",
                   help="HIP engine: run the periodic test-set eval on a side stream from a "
                        "parameter snapshot, overlapped with training (same accuracies)")
    p.add_argument("--no-native-exchange", action="store_true",
                   help="drive the sync exchange from Python instead of the C++ SyncRunner")
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--exchange", dest="exchange_backend", default=d.exchange_backend,
                   choices=["auto", "rccl", "xgmi"],
                   help="W > 1 sync data plane of the native runner: RCCL collectives or the "
                        "fused xGMI peer-memory exchange (flat plan)")
    p.add_argument("--log-jsonl", default=None)
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--checkpoint-every", type=int, default=0)
    p.add_argument("--resume", action="store_true",
                   help="continue from --checkpoint-dir: same data index, eval cadence and "
                        "dropout seeds as an uninterrupted run")
    p.add_argument("--max-steps", type=int, default=None,
                   help="stop after this many global steps (checkpointed if --checkpoint-dir)")
    p.add_argument("--target-acc", type=float, default=None)
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--watchdog-s", type=float, default=d.watchdog_s)
    return p


def from_args(a: argparse.Namespace) -> TrainConfig:
    mode, shard = a.mode, a.shard
    if a.variant:
        mode, shard = VARIANTS[a.variant]["mode"], VARIANTS[a.variant]["shard"]
    return TrainConfig(
        mode=mode, shard=shard, num_ps=a.num_ps, epochs=a.epochs, batch_size=a.batch_size,
        steps=a.steps, lr=a.lr, optimizer=a.optimizer, keep_prob=a.keep_prob,
        eval_every=a.eval_every, data=a.data, data_sharding=a.data_sharding,
        grad_reduce=a.grad_reduce, ref_quirks=a.ref_quirks, seed=a.seed, engine=a.engine,
        graph=a.graph and not a.no_graph, native_exchange=not a.no_native_exchange,
        dist_eval=not a.no_dist_eval, eval_async=a.eval_async,
        check_provenance=a.check_provenance, overlap=not a.no_overlap, log_jsonl=a.log_jsonl,
        exchange_backend=a.exchange_backend,
        checkpoint_dir=a.checkpoint_dir, checkpoint_every=a.checkpoint_every,
        resume=a.resume, max_steps=a.max_steps, target_acc=a.target_acc, quiet=a.quiet, watchdog_s=a.watchdog_s)
