#!/usr/bin/env python3
"""The strongest stock-PyTorch version of the benchmark step we can build on this image: the
reference CNN as nn modules in NCHW, MIOpen autotuning
(``cudnn.benchmark``), fused/capturable Adam, and the WHOLE training step (forward, backward,
optimizer) captured once as a HIP graph and replayed — no Python or launch overhead per step.
(No Triton on this image, so no torch.compile.)  Same shapes as bench.py: batch 100, fp32,
synthetic MNIST-shaped data; dropout keep 0.5.

Usage: python scripts/torch_best_baseline.py [--steps 200 --warmup 20]
Prints one JSON line per variant (eager, graph) with ms/step and images/s.
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class SamePool(nn.Module):
    def forward(self, h):
        if h.shape[-1] % 2:  # TF SAME: pad bottom/right (7 -> 4)
            h = F.pad(h, (0, 1, 0, 1), value=float("-inf"))
        return F.max_pool2d(h, 2, 2)


def model():
    layers = []
    cin = 1
    for cout in (32, 64, 128, 256):
        layers += [nn.Conv2d(cin, cout, 5, padding=2), nn.ReLU(), SamePool()]
        cin = cout
    layers += [nn.Flatten(), nn.Linear(1024, 1024), nn.ReLU(), nn.Dropout(0.5),
               nn.Linear(1024, 512), nn.Dropout(0.5), nn.Linear(512, 10)]
    return nn.Sequential(*layers)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=100)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = model().to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=1e-4, eps=1e-8, fused=True, capturable=True)
    x = torch.rand(50000, 1, 28, 28, device=dev)
    y = torch.randint(0, 10, (50000,), device=dev)
    B = a.batch
    sx = torch.empty(B, 1, 28, 28, device=dev)
    sy = torch.empty(B, dtype=torch.long, device=dev)

    def step():
        out = net(sx)
        loss = F.cross_entropy(out, sy)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        return loss

    def load(i):
        j = (i % (50000 // B)) * B
        sx.copy_(x[j:j + B])
        sy.copy_(y[j:j + B])

    res = {}
    # eager
    for i in range(a.warmup):
        load(i)
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        load(i)
        step()
    torch.cuda.synchronize()
    res["eager"] = 1e3 * (time.perf_counter() - t0) / a.steps

    # whole-step graph capture (warm up on a side stream first, as torch requires)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            load(i)
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for i in range(a.warmup):
        load(i)
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        load(i)
        g.replay()
    torch.cuda.synchronize()
    res["graph"] = 1e3 * (time.perf_counter() - t0) / a.steps
    for k, ms in res.items():
        print(json.dumps({"variant": f"stock-pytorch-{k}", "ms_per_step": round(ms, 4),
                          "images_per_s": round(B / ms * 1e3, 1), "batch": B,
                          "dtype": "fp32", "miopen_benchmark": True, "adam": "fused"}))


if __name__ == "__main__":
    main()
