#!/usr/bin/env python3
"""Run one GEMM op of the engine under one schedule many times (for a rocprofv3 --pmc pass):
where do a kernel's VALU instructions go — main loop, or per-block prologue / epilogue /
split-K bookkeeping that grows with the split factor?

usage: rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU ... -- \
           python3 scripts/pmc_sched_probe.py --op conv3_dgrad --cfg 3 --splits 8 [--workers 0] [--inline]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from op_bench import OPS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", required=True, choices=OPS)
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--inline", action="store_true", help="in-launch split-K reduce (mode 1)")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from ddl_amd.models.layout import CANON_OFFSETS, TOTAL_NUMEL
    from ddl_amd.models.mnist_cnn import init_params_
    from ddl_amd.models.hip_engine import HipEngine
    dev = torch.device("cuda")
    params = torch.zeros(TOTAL_NUMEL, device=dev)
    init_params_(params, CANON_OFFSETS, 0)
    grads = torch.zeros_like(params)
    eng = HipEngine(params, grads, CANON_OFFSETS, batch=100, graph=False, eval_chunk=100)
    x = torch.rand(100, 784, device=dev)
    y = torch.randint(0, 10, (100,), device=dev)
    seed = torch.tensor([7], dtype=torch.int32, device=dev)
    eng.forward_backward(x, y, 0.5, 7)
    op = OPS.index(a.op)
    cfg, spl, wk, wd = eng.get_cfg(), eng.get_splits(), eng.get_workers(), eng.eng.get_wide()
    cfg[op], spl[op], wk[op] = a.cfg, a.splits, a.workers
    wd[op] = (1 << 20) if a.inline else 1
    eng.set_cfg(cfg)
    eng.set_splits(spl)
    eng.set_workers(wk)
    eng.eng.set_wide(wd)
    torch.cuda.synchronize()
    for _ in range(a.iters):
        eng.eng.run_op(op, x, seed, True)
    torch.cuda.synchronize()
    print("done", a)


if __name__ == "__main__":
    main()
