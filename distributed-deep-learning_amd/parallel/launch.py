"""Process entry point: ``python -m ddl_amd.parallel.launch [flags]`` (one per GPU).

Reference launcher (``mnist_sync_sharding/run.sh:3``) is MPMD:
``mpiexec -n P python3 parameter_server.py -np P : -n W python3 worker.py -np W`` —
P PS processes plus W worker processes.  MI355X mapping: W processes (one per GPU,
``torchrun --nproc-per-node W``), the P PS roles co-located in them (PS p on rank
p % W).  ``run.sh <num_ps> <num_workers>`` at the repo root does that mapping.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

from ..config import add_args, from_args


def main(argv=None, mode_default: str = "sync") -> dict:
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    ap = add_args(argparse.ArgumentParser(description=__doc__), mode_default)
    ap.add_argument("--summary-json", default=None)
    a = ap.parse_args(argv)
    cfg = from_args(a)
    from .comm import init_distributed
    from .roles import Trainer
    env = init_distributed()
    if a.np_compat is not None and a.np_compat != env.world and env.rank == 0:
        # `worker.py -np W` (reference mnist_sync_sharding/worker.py:65): the worker count is
        # the launcher's process count here (parameter_server.py maps its -np to --num-ps)
        print(f"[ddl_amd] -np {a.np_compat} ignored: {env.world} worker process(es) were "
              f"launched (run.sh <num_ps> <num_workers> sets both)", file=sys.stderr)
    tr = Trainer(cfg, env)
    summary = tr.train()
    if a.summary_json and env.rank == 0:
        with open(a.summary_json, "w") as f:
            json.dump(summary, f, indent=1)
    if env.world > 1:
        import torch.distributed as dist
        from .roles import close_trainers
        close_trainers([tr], env)
        dist.destroy_process_group()
    return summary


if __name__ == "__main__":
    main(sys.argv[1:])
