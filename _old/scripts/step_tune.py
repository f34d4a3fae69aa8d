#!/usr/bin/env python3
"""Whole-step autotune of the HIP engine's per-op schedule (run on the GPU box).

Per-op sweeps (scripts/op_bench.py --json) time each GEMM alone; in the real step the
weight-gradient GEMMs run concurrently with the data-gradient GEMMs on a second stream, so
the best isolated schedule is not always the best in context.  This does coordinate descent
over each op's top candidates from the sweep, timing the full forward+backward step.

usage: python scripts/step_tune.py --sweep gpurun_out/op_sweep.json [--top 6] [--passes 2]
Prints DEFAULT_CFG / DEFAULT_SPLITS / DEFAULT_WORKERS for csrc/kernels/engine.hip.
"""
import argparse
import json
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from op_bench import OPS  # noqa: E402  (scripts/ is on sys.path when run as a script)


def parse_key(k):
    """c3s16 -> split-K 16 (separate reduce); c3s16m1 -> split-K 16 with the in-launch
    reduce (workers -1); c3w2048 -> stream-K 2048 workers."""
    m = re.fullmatch(r"c(\d+)([sw])(\d+)(m1)?", k)
    c, kind, v = int(m.group(1)), m.group(2), int(m.group(3))
    if kind == "w":
        return (c, 1, v)
    return (c, v, -1 if m.group(4) else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", required=True)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--concurrent", action="store_true", help="tune for the two-stream backward")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from ddl_amd.models.layout import CANON_OFFSETS, TOTAL_NUMEL
    from ddl_amd.models.mnist_cnn import init_params_
    from ddl_amd.models.hip_engine import HipEngine
    sweep = json.load(open(a.sweep))
    dev = torch.device("cuda")
    params = torch.zeros(TOTAL_NUMEL, device=dev)
    init_params_(params, CANON_OFFSETS, 0)
    grads = torch.zeros_like(params)
    B = a.batch
    eng = HipEngine(params, grads, CANON_OFFSETS, batch=B, graph=a.graph, eval_chunk=B)
    eng.set_concurrent(a.concurrent)
    x = torch.rand(B, 784, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)

    cands = {}
    for op, name in enumerate(OPS):
        us = sweep[name]["us"]
        ranked = sorted(us, key=us.get)[:a.top]
        cands[op] = [parse_key(k) for k in ranked]
    cfg, spl, wk = eng.get_cfg(), eng.get_splits(), eng.get_workers()
    default = (list(cfg), list(spl), list(wk))
    for op in range(len(OPS)):
        cfg[op], spl[op], wk[op] = cands[op][0]

    def apply():
        eng.set_cfg(cfg)
        eng.set_splits(spl)
        eng.set_workers([max(w, 0) for w in wk])
        eng.set_wide([1 << 20 if w < 0 else 1 for w in wk])

    def step_us():
        apply()
        for _ in range(5):
            eng.forward_backward(x, y, 0.5, 7)
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.iters):
                eng.forward_backward(x, y, 0.5, 7)
            en.record()
            torch.cuda.synchronize()
            best = min(best, 1e3 * st.elapsed_time(en) / a.iters)
        return best

    saved = (list(cfg), list(spl), list(wk))
    cfg[:], spl[:], wk[:] = default
    t_default = step_us()
    cfg[:], spl[:], wk[:] = saved
    cur = step_us()
    print(f"step default {t_default:.1f} us, per-op-best start {cur:.1f} us", flush=True)
    for p in range(a.passes):
        for op, name in enumerate(OPS):
            keep = (cfg[op], spl[op], wk[op])
            best_t, best_c = cur, keep
            for c in cands[op] + [(default[0][op], default[1][op], default[2][op])]:
                if c == keep:
                    continue
                cfg[op], spl[op], wk[op] = c
                t = step_us()
                if t < best_t * 0.995:
                    best_t, best_c = t, c
            cfg[op], spl[op], wk[op] = best_c
            cur = step_us()
            print(f"pass {p} {name:12s} -> c{best_c[0]} s{best_c[1]} w{best_c[2]}  step {cur:.1f} us",
                  flush=True)
    print("DEFAULT_CFG", ",".join(map(str, cfg)))
    print("DEFAULT_SPLITS", ",".join(map(str, spl)))
    print("DEFAULT_WORKERS", ",".join(str(max(w, 0)) for w in wk))
    print("DEFAULT_WIDE", ",".join(str(1 << 20 if w < 0 else 1) for w in wk))
    print(f"final step {cur:.1f} us (default {t_default:.1f} us)")
    if a.json:
        json.dump({"cfg": cfg, "splits": spl, "workers": [max(w, 0) for w in wk],
                   "wide": [1 << 20 if w < 0 else 1 for w in wk], "step_us": cur,
                   "default_step_us": t_default}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
