"""Multi-process helpers for the gloo (CPU) protocol tests: one spawned process per rank."""
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(rank, world, port):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)


def train_rank(rank, world, port, cfg_kw, outdir, n_train=600):
    """Run a Trainer for cfg_kw on this rank; save final params + PS step counters."""
    _setup(rank, world, port)
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed(device="cpu")
        cfg_kw = dict(cfg_kw)
        segs = cfg_kw.pop("_segments", None)
        if segs is not None:  # plan with another engine's backward segments (e.g. the HIP one's)
            import ddl_amd.parallel.roles as roles
            roles.engine_segments = lambda kind, device: segs
        cfg = TrainConfig(**cfg_kw)
        tr = Trainer(cfg, env, dataset=synthetic_mnist(n_train, 200, seed=7))
        summary = tr.train()
        torch.save({"params": tr.params.clone(), "plan_offsets": tr.plan.tensor_offsets,
                    "ps_t": {p: s.t for p, s in tr.servers.items()},
                    "num_ps": tr.num_ps,
                    "served": getattr(tr.exchange, "served", None),
                    "provenance": list(getattr(tr.exchange, "provenance", []) or []),
                    "summary": summary},
                   os.path.join(outdir, f"rank{rank}.pt"))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


def spawn(fn, world, *args):
    import torch.multiprocessing as mp
    mp.spawn(fn, args=(world, *args), nprocs=world, join=True)


def simulate_sync(cfg_kw, world, n_train=600):
    """Single-process model of synchronous PS training: every worker's gradient on its
    batch (own dropout seed), summed (x quirk coefficients), one Adam step per global step."""
    from ddl_amd.config import TrainConfig
    from ddl_amd.models.layout import CANON_OFFSETS, TOTAL_NUMEL
    from ddl_amd.models.mnist_cnn import TorchEngine, init_params_
    from ddl_amd.ops import rng
    from ddl_amd.ops.adam import AdamHyper, adam_torch_
    from ddl_amd.parallel.comm import quirk_coefficient
    from ddl_amd.parallel.sharding import make_plan
    from ddl_amd.utils.data import synthetic_mnist, batch_indices
    cfg = TrainConfig(**cfg_kw)
    data = synthetic_mnist(n_train, 200, seed=7)
    params = torch.zeros(TOTAL_NUMEL)
    init_params_(params, CANON_OFFSETS, cfg.seed)
    grads = torch.zeros_like(params)
    acc = torch.zeros_like(params)
    eng = TorchEngine(params, grads, CANON_OFFSETS, cfg.batch_size)
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    h = AdamHyper(lr=cfg.lr)
    num_ps = 1 if cfg.shard == "none" else (cfg.num_ps or world)
    plan = make_plan(cfg.shard, num_ps)
    steps = cfg.steps * cfg.epochs
    worker_init = None
    if cfg.ref_quirks and world > 1:
        # Q4: every process initialises independently (seed + rank).  A sync PS updates its
        # host's buffer in place, so the PS state starts as each tensor's host's init, while
        # the step-0 gradients are computed by every worker at its OWN init
        # (mnist_sync/parameter_server.py:17-18,31; mnist_sync/model/model.py:112).
        from ddl_amd.models.layout import TENSORS
        if not plan.tensor_granular:
            raise NotImplementedError("quirk simulation covers the tensor-granular plans")
        worker_init = []
        for r in range(world):
            p_r = torch.zeros(TOTAL_NUMEL)
            init_params_(p_r, CANON_OFFSETS, cfg.seed + r)
            worker_init.append(p_r)
        for t in TENSORS:
            host = plan.host_rank(plan.owner[t.index], world)
            o = CANON_OFFSETS[t.index]
            params[o:o + t.numel] = worker_init[host][o:o + t.numel]
    for step in range(steps):
        acc.zero_()
        ps_params = params.clone() if (worker_init is not None and step == 0) else None
        for r in range(world):
            if ps_params is not None:
                params.copy_(worker_init[r])
            lo, hi = batch_indices(step % cfg.steps, cfg.batch_size, data.total_batch, r, world,
                                   cfg.data_sharding)
            eng.forward_backward(data.x_train[lo:hi], data.y_train[lo:hi], cfg.keep_prob,
                                 rng.step_seed(cfg.seed, r, step))
            acc.add_(grads, alpha=quirk_coefficient(plan, r, world, cfg.ref_quirks))
        if ps_params is not None:
            params.copy_(ps_params)
        if cfg.grad_reduce == "mean":
            acc.div_(world)
        adam_torch_(params, acc, m, v, h, step + 1)
    return params


def eval_rank(rank, world, port, outdir):
    """Distributed (1/W per rank + all-reduce) vs full test-set accuracy after a few steps."""
    _setup(rank, world, port)
    try:
        import torch.distributed as dist
        from ddl_amd.config import TrainConfig
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.roles import Trainer
        from ddl_amd.utils.data import synthetic_mnist
        env = init_distributed(device="cpu")
        tr = Trainer(TrainConfig(mode="sync", shard="contiguous", steps=3, eval_every=0,
                                 quiet=True), env, dataset=synthetic_mnist(600, 301, seed=9))
        for i in range(3):
            tr.train_step(i)
        dist_acc = tr.evaluate()
        tr.cfg.dist_eval = False
        full_acc = tr.evaluate()
        torch.save({"dist": dist_acc, "full": full_acc}, os.path.join(outdir, f"eval{rank}.pt"))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise


def handoff_vote_rank(rank, world, port, outdir, case):
    """One rank of the hand-off vote (native_exchange.handoff_vote) over gloo: `case` names the
    digests this rank reports; the verdict (or the refusal) is saved per rank."""
    _setup(rank, world, port)
    try:
        import torch.distributed as dist
        from ddl_amd.parallel.comm import init_distributed
        from ddl_amd.parallel.native_exchange import NativeUnavailable, handoff_vote
        env = init_distributed(device="cpu")
        ev, fl = "a" * 64, "a" * 64
        if case == "replicas_diverge" and rank == world - 1:
            ev = fl = "b" * 64      # this rank's replica differs under both hand-offs
        elif case == "flags_diverge" and rank == world - 1:
            fl = "c" * 64           # only the READY-flag run differs
        try:
            out = handoff_vote(env, ev, fl)
        except NativeUnavailable as e:
            out = {"refused": str(e)}
        torch.save(out, os.path.join(outdir, f"rank{rank}.pt"))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        traceback.print_exc()
        raise
