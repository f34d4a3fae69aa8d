#!/usr/bin/env python3
"""conv2 weight-gradient error vs fp64 across split-K / stream-K schedules (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from ddl_amd.models.layout import TENSORS, CANON_OFFSETS, TOTAL_NUMEL  # noqa: E402
from ddl_amd.models.mnist_cnn import init_params_, param_views, torch_forward, xent_loss  # noqa: E402
from ddl_amd.models.hip_engine import HipEngine  # noqa: E402

OP = 15  # OP_CONV2_WGRAD


def main():
    torch.manual_seed(0)
    flat = torch.zeros(TOTAL_NUMEL)
    init_params_(flat, CANON_OFFSETS, seed=3)
    for t, v in zip(TENSORS, param_views(flat, CANON_OFFSETS)):
        if t.kind == "bias":
            v.add_(torch.randn_like(v) * 0.05)
    params = flat.cuda()
    grads = torch.zeros_like(params)
    eng = HipEngine(params, grads, CANON_OFFSETS, batch=100, graph=False, eval_chunk=500)
    x = torch.rand(100, 784)
    y = torch.randint(0, 10, (100,))
    pv = [v.detach().double().clone().requires_grad_(True) for v in param_views(flat, CANON_OFFSETS)]
    loss = xent_loss(torch_forward(pv, x.double(), 0.5, 99), y)
    r64 = torch.autograd.grad(loss, pv)
    pv32 = [v.detach().clone().requires_grad_(True) for v in param_views(flat, CANON_OFFSETS)]
    r32 = torch.autograd.grad(xent_loss(torch_forward(pv32, x, 0.5, 99), y), pv32)
    o, n = CANON_OFFSETS[2], TENSORS[2].numel
    ref = r64[2].reshape(-1)
    e32 = float((r32[2].reshape(-1).double() - ref).abs().max() / ref.abs().max())
    print(f"torch fp32 CPU vs fp64: {e32:.3e}   max|ref| {float(ref.abs().max()):.3e}")
    base_c, base_s, base_w, base_wd = eng.get_cfg(), eng.get_splits(), eng.get_workers(), eng.get_wide()
    for c in (3, 4):
        for s in (1, 8, 16, 32, 64, 128, 256):
            for wd in (1, 1 << 20):
                cf, sp, wk, wde = list(base_c), list(base_s), list(base_w), list(base_wd)
                cf[OP], sp[OP], wk[OP], wde[OP] = c, s, 0, wd
                eng.set_cfg(cf); eng.set_splits(sp); eng.set_workers(wk); eng.set_wide(wde)
                grads.zero_()
                eng.forward_backward(x.cuda(), y.cuda(), 0.5, 99)
                torch.cuda.synchronize()
                g = grads[o:o + n].double().cpu()
                err = float((g - ref).abs().max() / ref.abs().max())
                arg = int((g - ref).abs().argmax())
                print(f"c{c} s{s:4d} {'inlaunch' if wd > 1 else 'separate'}: err {err:.3e} at {arg} "
                      f"(got {float(g[arg]):.4e} ref {float(ref[arg]):.4e})", flush=True)


if __name__ == "__main__":
    main()
