#!/usr/bin/env python3
"""Per-tensor gradient error vs fp64 under several engine schedules (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.models.layout import TENSORS, CANON_OFFSETS, TOTAL_NUMEL  # noqa: E402
from ddl_amd.models.mnist_cnn import init_params_, param_views, torch_forward, xent_loss  # noqa: E402
from ddl_amd.models.hip_engine import HipEngine  # noqa: E402


def main():
    torch.manual_seed(0)
    flat = torch.zeros(TOTAL_NUMEL)
    init_params_(flat, CANON_OFFSETS, seed=3)
    params = flat.cuda()
    grads = torch.zeros_like(params)
    eng = HipEngine(params, grads, CANON_OFFSETS, batch=100, graph=False, eval_chunk=500)
    x = torch.rand(100, 784)
    y = torch.randint(0, 10, (100,))
    pv = [v.detach().double().clone().requires_grad_(True) for v in param_views(flat, CANON_OFFSETS)]
    r64 = torch.autograd.grad(xent_loss(torch_forward(pv, x.double(), 0.5, 5), y), pv)
    n = len(eng.get_cfg())
    base = (eng.get_cfg(), eng.get_splits(), eng.get_workers(), eng.get_wide())
    variants = {"default": base, "nodual": base}
    for c in (0, 1, 2, 3, 4):
        for sp in (1, 4):
            variants[f"split{sp}_cfg{c}"] = ([c] * n, [sp] * n, [0] * n, [1] * n)
    variants["sk1024_cfg0"] = ([0] * n, [1] * n, [1024] * n, [1] * n)
    for name, (c, s, w, wd) in variants.items():
        eng.set_cfg(c); eng.set_splits(s); eng.set_workers(w); eng.set_wide(wd)
        eng.set_dual(name != "nodual")
        grads.zero_()
        eng.forward_backward(x.cuda(), y.cuda(), 0.5, 5)
        torch.cuda.synchronize()
        errs = []
        for t, g in zip(TENSORS, param_views(grads, CANON_OFFSETS)):
            ref = r64[t.index]
            errs.append(float((g.double().cpu() - ref).abs().max() / ref.abs().max()))
        print(f"{name:14s} " + " ".join(f"{e:8.1e}" for e in errs), flush=True)


if __name__ == "__main__":
    main()
