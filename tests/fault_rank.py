"""One rank of a fault-injection job (tests/test_fault_injection_cpu.py, test_xgmi_gpu.py).

    python tests/fault_rank.py RANK WORLD PORT DEVICE FAULT OUTDIR

DEVICE: ``cpu`` (gloo, torch engine) or ``xgmi`` (one GPU shared by every rank, gloo default
group, the native xGMI exchange).  FAULT: ``kill@R:S`` (rank R leaves with os._exit(17) at the
start of its step S — a crashed process), ``stop@R:S`` (rank R SIGSTOPs itself there — a hung
one), or ``none``.  Each surviving rank writes ``OUTDIR/rank{r}.exit`` with the exception it
saw (if any) just before the process ends; the exit status and the wall time are what the
tests check: a survivor must END, non-zero, within the watchdog bound (the
reference's blocking loop ``mnist_sync/parameter_server.py:57-69`` waits forever instead).
"""
import os
import signal
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    device, fault, outdir = sys.argv[4], sys.argv[5], sys.argv[6]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if device == "xgmi":
        os.environ.update(DDL_DIST_BACKEND="gloo", DDL_XGMI_TIMEOUT_S="4")
    import torch
    torch.set_num_threads(1)
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import init_distributed
    from ddl_amd.parallel import roles
    from ddl_amd.utils.data import synthetic_mnist

    steps = int(os.environ.get("DDL_FAULT_STEPS", "400"))  # long enough to be mid-run
    kind, where = (fault.split("@") + [""])[:2]
    f_rank, f_step = (int(v) for v in where.split(":")) if where else (-1, -1)
    orig = roles.Trainer.train_step

    def faulty(self, step):
        if self.env.rank == f_rank and self.global_step == f_step:
            sys.stdout.flush()
            if kind == "kill":
                os._exit(17)
            if kind == "stop":
                os.kill(os.getpid(), signal.SIGSTOP)
        return orig(self, step)

    roles.Trainer.train_step = faulty
    note = os.path.join(outdir, f"rank{rank}.exit")
    try:
        if device == "cpu":
            env = init_distributed(device="cpu")
            cfg = TrainConfig(mode="sync", shard="contiguous", steps=steps, batch_size=10,
                              eval_every=0, quiet=True, engine="torch", watchdog_s=6.0)
        else:
            env = init_distributed()
            cfg = TrainConfig(mode="sync", shard="flat", steps=steps, batch_size=100,
                              eval_every=0, quiet=True, engine="hip", watchdog_s=12.0,
                              data_sharding="stride", exchange_backend="xgmi")
        tr = roles.Trainer(cfg, env, dataset=synthetic_mnist(4000, 100, seed=3))
        tr.train()
    except BaseException:
        with open(note, "w") as f:
            f.write(traceback.format_exc())
        sys.stderr.write(traceback.format_exc())
        sys.stderr.flush()
        os._exit(3)  # no interpreter teardown: a dead peer's process group may block in it
    with open(note, "w") as f:
        f.write("completed\n")
    os._exit(0)


if __name__ == "__main__":
    main()
