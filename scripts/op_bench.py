#!/usr/bin/env python3
"""Per-op timing of the HIP engine's GEMM ops and split-K sweep (run on the GPU box).

usage: python scripts/op_bench.py [--batch 100] [--iters 50] [--splits 1,2,4,8,16]
Prints one line per (op, split): mean us per launch (device events), plus the step total.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = ["conv1_fwd", "conv2_fwd", "conv3_fwd", "conv4_fwd", "fc1_fwd", "fc2_fwd",
       "fc2_dgrad", "fc2_wgrad", "fc1_dgrad", "fc1_wgrad", "conv4_dgrad", "conv4_wgrad",
       "conv3_dgrad", "conv3_wgrad", "conv2_dgrad", "conv2_wgrad", "conv1_wgrad"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--splits", default="1,2,4,8,16,32")
    ap.add_argument("--cfgs", default="0,1,2,3")
    ap.add_argument("--workers", default="0", help="stream-K worker counts to sweep (0 = none)")
    ap.add_argument("--m1-max", type=int, default=32,
                    help="also sweep split-K with the in-launch reduce for splits <= this")
    ap.add_argument("--json", default=None)
    ap.add_argument("--ops", default="", help="comma-separated op names (default: all)")
    ap.add_argument("--no-step", action="store_true", help="skip the whole-step timing")
    a = ap.parse_args()
    from ddl_amd.models.layout import CANON_OFFSETS, TOTAL_NUMEL
    from ddl_amd.models.mnist_cnn import init_params_
    from ddl_amd.models.hip_engine import HipEngine
    dev = torch.device("cuda")
    params = torch.zeros(TOTAL_NUMEL, device=dev)
    init_params_(params, CANON_OFFSETS, 0)
    grads = torch.zeros_like(params)
    B = a.batch
    eng = HipEngine(params, grads, CANON_OFFSETS, batch=B, graph=False, eval_chunk=B)
    x = torch.rand(B, 784, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    seed = torch.tensor([7], dtype=torch.int32, device=dev)
    base = eng.get_splits()
    eng.forward_backward(x, y, 0.5, 7)
    torch.cuda.synchronize()

    def time_op(op, iters):
        for _ in range(3):
            eng.eng.run_op(op, x, seed, True)
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(iters):
            eng.eng.run_op(op, x, seed, True)
        en.record()
        torch.cuda.synchronize()
        return 1e3 * st.elapsed_time(en) / iters

    res = {}
    sweep = [int(s) for s in a.splits.split(",")]
    wsweep = [int(w) for w in a.workers.split(",") if int(w) > 0]
    cfgs = [int(c) for c in a.cfgs.split(",")]
    base_cfg = eng.get_cfg()
    base_w = eng.get_workers()
    best_cfg, best_split, best_w = list(base_cfg), list(base), list(base_w)
    only = set(a.ops.split(",")) if a.ops else None
    for op, name in enumerate(OPS):
        if only is not None and name not in only:
            continue
        M, N, K = eng.eng.op_shape(op, B)
        flop = 2.0 * M * N * K
        row = {}
        # (cfg, splits, workers): split-K points have workers 0, stream-K points splits 1
        # (cfg, splits, workers): split-K points have workers 0 (workers -1: split-K with the
        # in-launch last-arriver reduce), stream-K points splits 1
        points = ([(c, s, 0) for c in cfgs for s in sweep]
                  + [(c, s, -1) for c in cfgs for s in sweep if 1 < s <= a.m1_max]
                  + [(c, 1, w) for c in cfgs for w in wsweep])
        base_wide = eng.get_wide()
        for c, s, w in points:
            cf, sp, wk, wd = list(base_cfg), list(base), list(base_w), list(base_wide)
            cf[op], sp[op], wk[op] = c, s, max(w, 0)
            wd[op] = 1 << 20 if w < 0 else 1
            eng.set_splits(sp)
            eng.set_cfg(cf)
            eng.set_workers(wk)
            eng.set_wide(wd)
            row[(c, s, w)] = time_op(op, a.iters)
        eng.set_splits(base)
        eng.set_cfg(base_cfg)
        eng.set_workers(base_w)
        eng.set_wide(base_wide)
        best = min(row, key=row.get)
        best_cfg[op], best_split[op], best_w[op] = best[0], best[1], best[2]
        key = lambda t: (f"c{t[0]}w{t[2]}" if t[2] > 0 else
                         f"c{t[0]}s{t[1]}m1" if t[2] < 0 else f"c{t[0]}s{t[1]}")
        dflt = (base_cfg[op], base[op] if not base_w[op] else 1, base_w[op])
        res[name] = {"M": M, "N": N, "K": K, "us": {key(t): v for t, v in row.items()},
                     "best": key(best), "best_us": row[best],
                     "default_us": row.get(dflt),
                     "best_tflops": flop / row[best] / 1e6}
        print(f"{name:12s} M={M:6d} N={N:5d} K={K:6d} default {key(dflt)}="
              f"{row.get(dflt, float('nan')):7.1f}  best {key(best)}="
              f"{row[best]:7.1f} us {flop / row[best] / 1e6:6.1f} TF", flush=True)
        for c in cfgs:
            print("      c%d " % c + " ".join(f"{key(t)[len(str(c)) + 1:]}:{v:7.1f}"
                                          for t, v in row.items() if t[0] == c), flush=True)
    print("BEST_CFG", ",".join(map(str, best_cfg)))
    print("BEST_SPLITS", ",".join(map(str, best_split)))
    best_wide = [1 << 20 if w < 0 else 1 for w in best_w]
    best_w = [max(w, 0) for w in best_w]
    print("BEST_WORKERS", ",".join(map(str, best_w)))
    print("BEST_WIDE", ",".join(map(str, best_wide)))
    eng.set_cfg(best_cfg)
    eng.set_splits(best_split)
    eng.set_workers(best_w)
    eng.set_wide(best_wide)
    # whole step eager vs graph
    for g in ((False, True) if not a.no_step else ()):
        e2 = HipEngine(params, grads, CANON_OFFSETS, batch=B, graph=g, eval_chunk=B)
        e2.set_concurrent(False)
        e2.set_cfg(best_cfg)
        e2.set_splits(best_split)
        e2.set_workers(best_w)
        e2.set_wide(best_wide)
        for _ in range(5):
            e2.forward_backward(x, y, 0.5, 7)
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(a.iters):
            e2.forward_backward(x, y, 0.5, 7)
        en.record()
        torch.cuda.synchronize()
        print(f"fwd+bwd step graph={g}: {1e3 * st.elapsed_time(en) / a.iters:.1f} us", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
