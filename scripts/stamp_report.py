#!/usr/bin/env python3
"""Per-block timeline report of the conv backward dual launches (diagnostic stamp build).

    DDL_BUILD_TAG=stamp DDL_EXTRA_CFLAGS=-DDDL_STAMPS=1 python build.py     # here, on the CPU
    DDL_SO=_C_stamp.so python scripts/stamp_report.py [--sched tuned.json]  # on the GPU box

Runs the default native-runner step, then records STEPS steps with every split-K block of the
dual launches stamping its start / end (100 MHz constant clock and shader clock), the hardware
slot it ran on and its K-tile count (csrc/kernels/stamps.h).  Per launch and sub-problem: span,
block-length spread, time per K tile, start skew, the tail after 90 % of the blocks have
finished, waves per SIMD over the span (occupancy of the hardware slots) and the clock.
"""
import argparse
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--sched", default=None, help="a runner_tune.py JSON schedule")
    ap.add_argument("--json", default=None)
    ap.add_argument("--nodual", action="store_true", help="data / weight gradients back to back")
    a = ap.parse_args()
    import torch
    from ddl_amd.config import TrainConfig
    from ddl_amd.ops import native
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import synthetic_mnist

    C = native.ops()
    assert C.stamps_enabled(), "load the stamp build: DDL_SO=_C_stamp.so"
    tr = Trainer(TrainConfig(mode="sync", shard="flat", steps=10 ** 6, eval_every=0, engine="hip",
                             quiet=True), DistEnv(0, 1, 0, torch.device("cuda", 0)),
                 dataset=synthetic_mnist(n_train=5000, n_test=500))
    e = tr.engine.eng
    if a.sched:
        sc = json.load(open(a.sched))
        e.set_cfg(sc["cfg"]), e.set_splits(sc["splits"])
        e.set_wide(sc["wide"])
    if a.nodual:
        e.set_dual(False)
    for i in range(60):
        tr.train_step(i)
    torch.cuda.synchronize()
    C.stamps_begin(1 << 17)
    for i in range(a.steps):
        tr.train_step(60 + i)
    rec, log = C.stamps_end()
    rec = rec.tolist()
    cfg = e.get_cfg()
    # group the sub-grids into launches: (sub 0, sub 1) = a dual launch, sub 2 = a single one
    launches, i = [], 0
    while i < len(log):
        if log[i][2] == 0 and i + 1 < len(log) and log[i + 1][2] == 1:
            launches.append(log[i:i + 2])
            i += 2
        else:
            launches.append(log[i:i + 1])
            i += 1
    per_step = len(launches) // a.steps
    names = (["conv2_fwd", "conv3_fwd", "conv4_fwd", "fc2_fwd", "conv4_bwd", "conv3_bwd",
              "conv2_bwd"] if per_step == 7 else [f"L{j}" for j in range(per_step)])
    print(f"{len(log)} sub-grids, {len(launches)} launches over {a.steps} steps; cfg {cfg}")
    print(f"{'launch':9s} {'sub':3s} {'blocks':>6s} {'span':>6s} {'blk med':>7s} {'blk p10':>7s} "
          f"{'blk max':>7s} {'us/kt':>6s} {'kt med':>6s} {'kt max':>6s} {'start90':>7s} "
          f"{'tail10':>6s} {'w/SIMD':>6s} {'maxres':>6s} {'GHz':>5s}")
    out = []
    for li, group in enumerate(launches):
        blocks_all = []
        for (off, nb, sub, gx, gy, gz) in group:
            blocks_all += rec[off:off + nb]
        t0 = min(r[0] for r in blocks_all)
        t1 = max(r[1] for r in blocks_all)
        span = (t1 - t0) / 100.0  # us
        simd_busy = defaultdict(float)
        ev = defaultdict(list)
        for r in blocks_all:
            hw, xcc = r[4] & 0xffffffff, r[4] >> 32
            key = (xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15, (hw >> 4) & 3)
            simd_busy[key] += (r[1] - r[0]) / 100.0
            ev[key] += [(r[0], 1), (r[1], -1)]
        maxres = 0
        for key, es in ev.items():  # most blocks resident at once on one SIMD
            c = 0
            for _, d in sorted(es, key=lambda x: (x[0], x[1])):
                c += d
                maxres = max(maxres, c)
        nsimd = len(simd_busy)
        wps = sum(simd_busy.values()) / max(1, nsimd) / span if span else 0
        for (off, nb, sub, gx, gy, gz) in group:
            rs = rec[off:off + nb]
            d = [(r[1] - r[0]) / 100.0 for r in rs]
            kt = [r[5] & 0xfffff for r in rs]
            last = [(r[5] >> 20) & 1 for r in rs]
            # block time = fixed + per_kt * K tiles (least squares over the blocks that did not
            # run the epilogue, i.e. stored a partial and left) and the epilogue blocks' extra
            fit = None
            xs = [k for k, l in zip(kt, last) if not l]
            ys = [t for t, l in zip(d, last) if not l]
            if len(set(xs)) > 1:
                n = len(xs)
                mx, my = sum(xs) / n, sum(ys) / n
                sxx = sum((x - mx) ** 2 for x in xs)
                b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx
                fit = (my - b * mx, b)
            ep = [t for t, l in zip(d, last) if l]
            # phases (diagnostic build with mid stamps): main loop, partial + ticket, epilogue
            loop = [(r[2] - r[0]) / 100.0 for r in rs if r[2] > r[0]]
            tick = [(r[3] - r[2]) / 100.0 for r in rs if r[3] > r[2] > 0]
            epil = [(r[1] - r[3]) / 100.0 for r, l in zip(rs, last) if l and r[3] > 0]
            us_kt = [x / max(1, k) for x, k in zip(d, kt)]
            starts = [(r[0] - t0) / 100.0 for r in rs]
            ends = sorted((r[1] - t0) / 100.0 for r in rs)
            ghz = [0.0]  # (r[2], r[3] hold the phase stamps now, not the shader clock)
            row = dict(launch=names[li % per_step], step=li // per_step, sub=sub, blocks=nb,
                       span=span, blk_med=pct(d, .5), blk_p10=pct(d, .1), blk_max=max(d),
                       us_per_kt=pct(us_kt, .5), kt_med=pct(kt, .5), kt_max=max(kt),
                       start90=pct(starts, .9), tail10=span - pct(ends, .9), waves_per_simd=wps,
                       max_resident=maxres, simds=nsimd, ghz=pct(ghz, .5),
                       fixed_us=fit[0] if fit else None, per_kt_us=fit[1] if fit else None,
                       epi_blocks=len(ep), epi_med=pct(ep, .5) if ep else None,
                       loop_med=pct(loop, .5) if loop else None,
                       ticket_med=pct(tick, .5) if tick else None,
                       epilogue_med=pct(epil, .5) if epil else None)
            out.append(row)
            print(f"{row['launch']:9s} {sub:3d} {nb:6d} {span:6.1f} {row['blk_med']:7.1f} "
                  f"{row['blk_p10']:7.1f} {row['blk_max']:7.1f} {row['us_per_kt']:6.2f} "
                  f"{row['kt_med']:6d} {row['kt_max']:6d} {row['start90']:7.1f} "
                  f"{row['tail10']:6.1f} {wps:6.2f} {maxres:6d} {row['ghz']:5.2f}"
                  + (f"  fit {fit[0]:5.2f} + {fit[1]:5.2f}/kt" if fit else "  fit -")
                  + (f"  epi {len(ep)} med {row['epi_med']:5.1f}" if ep else "")
                  + (f"  phases loop {row['loop_med']:5.1f}" if loop else "")
                  + (f" ticket {row['ticket_med']:4.1f}" if tick else "")
                  + (f" epi {row['epilogue_med']:4.1f}" if epil else ""))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
        # the last step's raw records (one row per block: stamps.h layout) + sub-grid table
        import numpy as np
        last = [x for g in launches[-per_step:] for x in g]
        lo = last[0][0]
        hi = last[-1][0] + last[-1][1]
        np.savez(a.json.replace(".json", "_raw.npz"), rec=np.array(rec[lo:hi], dtype=np.int64),
                 log=np.array([[x[0] - lo] + list(x[1:]) for x in last], dtype=np.int64))


if __name__ == "__main__":
    main()
