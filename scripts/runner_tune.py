#!/usr/bin/env python3
"""Coordinate-descent schedule tune on the REAL training step (native runner, W = 1: dual
launches, optimizer tail, fused end-of-backward launch) — unlike step_tune.py, which times the
Python engine path.  Per op, candidates around the current schedule (split x0.5 / x2, in-launch
vs separate reduce, stream-K worker counts, tile config 3 / 5); a candidate is kept only if it
beats the incumbent by > --gain in a re-measured head-to-head.

usage: python scripts/runner_tune.py [--passes 2] [--steps 250] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# engine op order (csrc/kernels/api.h enum Op)
OPS = ["conv1_fwd", "conv2_fwd", "conv3_fwd", "conv4_fwd", "fc1_fwd", "fc2_fwd",
       "fc2_dgrad", "fc2_wgrad", "fc1_dgrad", "fc1_wgrad", "conv4_dgrad", "conv4_wgrad",
       "conv3_dgrad", "conv3_wgrad", "conv2_dgrad", "conv2_wgrad", "conv1_wgrad"]

KWAVE_OK = {4, 5, 6, 8}  # fc forward / data-gradient GEMMs (csrc/kernels/layers.h KWaveOK)
MF16_OK = {1, 2, 3, 10, 11, 12, 13, 14, 15}  # conv GEMMs with 16-byte gathers (layers.h Mf16OK)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=250)
    ap.add_argument("--gain", type=float, default=0.004)
    ap.add_argument("--json", default=None)
    ap.add_argument("--ops", default=None, help="comma-separated op indices to tune (default all)")
    ap.add_argument("--multiwave", action="store_true",
                    help="also try the multi-wave block tiles (configs 1, 2, 6, 7, 8) on the "
                         "forward convolutions (not dual-launched, so any tile config runs)")
    ap.add_argument("--verbose", action="store_true", help="print every candidate's time")
    ap.add_argument("--dma", action="store_true",
                    help="also try the 16x16x4 tile (config 14) at 0.5x and 4x the split")
    a = ap.parse_args()
    import torch
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import synthetic_mnist

    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", shard="flat", steps=10 ** 7, batch_size=100, eval_every=0,
                      engine="hip", quiet=True, data_sharding="stride")
    tr = Trainer(cfg, env, dataset=synthetic_mnist())
    e = tr.engine.eng
    W = 1 << 20
    cur = {"cfg": e.get_cfg(), "splits": e.get_splits(), "wide": e.get_wide()}
    step = [0]

    def apply(s):
        e.set_cfg(s["cfg"])
        e.set_splits(s["splits"])
        e.set_wide(s["wide"])

    def timed(s):
        apply(s)
        for _ in range(20):
            tr.train_step(step[0])
            step[0] += 1
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tr.train_step(step[0])
            step[0] += 1
        torch.cuda.synchronize()
        return 1e6 * (time.perf_counter() - t0) / a.steps

    def cands(op):
        c, s, wd = cur["cfg"][op], cur["splits"][op], cur["wide"][op]
        out = []

        def mk(c2, s2, _w, wd2):
            d = {k: list(v) for k, v in cur.items()}
            d["cfg"][op], d["splits"][op], d["wide"][op] = c2, s2, wd2
            return d
        # x0.5 / x2, and the neighbours (+-1, x0.75 / x1.5) for a fine pass
        for s2 in sorted({max(1, s // 2), min(2048, s * 2), max(1, s - 1), s + 1,
                          max(1, (3 * s) // 4), min(2048, (3 * s) // 2)} - {s}):
            out.append(mk(c, s2, 0, wd))
        out.append(mk(c, s, 0, 1 if wd > 1 else W))            # toggle the reduce mode
        for c2 in (0, 3, 4, 5):  # the one-wave configs (dual launches instantiate these)
            if c2 != c:
                out.append(mk(c2, s, 0, wd))
        if op in MF16_OK:  # CFG_MF16 (16x16x4 MFMA, LDS-DMA), at the split and twice it
            for s2 in sorted({s, min(2048, s * 2)}):
                if (c, s) != (14, s2):
                    out.append(mk(14, s2, 0, wd))
        if op in MF16_OK and a.dma:  # (configs 16-20 were removed in round 6)
            for s2 in sorted({min(2048, s * 4), max(1, s // 2)}):
                if (c, s) != (14, s2):
                    out.append(mk(14, s2, 0, wd))
        if a.multiwave and op in (0, 1, 2, 3):
            for c2 in (1, 2, 6, 7, 8):
                for s2 in sorted({s, min(2048, s * 2), max(1, s // 2)}):
                    out.append(mk(c2, s2, 0, wd))
        if op in KWAVE_OK:  # K split over the waves of one workgroup (4 / 8 / 16 waves)
            for s2 in (4, 8, 16):
                if (c, s) != (13, s2):
                    out.append(mk(13, s2, 0, wd))
        return out

    base = timed(cur)
    print(f"start {base:.1f} us/step", flush=True)
    for p in range(a.passes):
        for op, name in enumerate(OPS):
            if a.ops and op not in {int(o) for o in a.ops.split(",")}:
                continue
            best, best_t = None, None
            for cand in cands(op):
                t = timed(cand)
                if a.verbose:
                    print(f"    {name:12s} c{cand['cfg'][op]} s{cand['splits'][op]} "
                          f"{'inl' if cand['wide'][op] > 1 else 'wide'} "
                          f"{t:.1f}", flush=True)
                if best_t is None or t < best_t:
                    best, best_t = cand, t
            # head-to-head re-measure of the incumbent vs the best candidate
            t_inc = min(timed(cur), timed(cur))
            t_new = min(timed(best), timed(best))
            if t_new < t_inc * (1 - a.gain):
                cur = best
                print(f"pass {p} {name:12s} -> c{cur['cfg'][op]} s{cur['splits'][op]} "
                      f"{'inl' if cur['wide'][op] > 1 else 'wide'}  "
                      f"{t_inc:.1f} -> {t_new:.1f} us", flush=True)
            else:
                print(f"pass {p} {name:12s} keep ({t_inc:.1f} vs best cand {t_new:.1f})", flush=True)
    final = min(timed(cur), timed(cur))
    print(f"final {final:.1f} us/step (start {base:.1f})")
    print("DEFAULT_CFG", ",".join(map(str, cur["cfg"])))
    print("DEFAULT_SPLITS", ",".join(map(str, cur["splits"])))
    print("DEFAULT_INL", ",".join("1" if w > 1 else "0" for w in cur["wide"]))
    if a.json:
        json.dump(dict(cur, step_us=final, start_us=base), open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
