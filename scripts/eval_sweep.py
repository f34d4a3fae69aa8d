#!/usr/bin/env python3
"""Tune the eval forward (full 10k test-set accuracy, the reference's every-10-steps eval that
dominates time-to-accuracy): test-set chunk size x per-op tile config, coordinate descent on
the measured full-eval time.

usage: python scripts/eval_sweep.py [--chunks 2000,5000,10000] [--cfgs 0,1,2,3,4,6,7,8]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="2000,5000,10000")
    ap.add_argument("--cfgs", default="0,1,2,3,4,6,7,8,9,10,11,12")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from ddl_amd.models.layout import CANON_OFFSETS, TOTAL_NUMEL
    from ddl_amd.models.mnist_cnn import init_params_
    from ddl_amd.models.hip_engine import HipEngine
    from ddl_amd.utils.data import synthetic_mnist

    dev = torch.device("cuda")
    params = torch.zeros(TOTAL_NUMEL, device=dev)
    init_params_(params, CANON_OFFSETS, 0)
    grads = torch.zeros_like(params)
    data = synthetic_mnist()
    x, y = data.x_test.to(dev), data.y_test.to(dev)
    cfgs = [int(c) for c in a.cfgs.split(",")]
    best_all = None
    for chunk in [int(c) for c in a.chunks.split(",")]:
        eng = HipEngine(params, grads, CANON_OFFSETS, batch=100, graph=False, eval_chunk=chunk)
        ref = eng.correct(x, y)

        def t_eval():
            for _ in range(2):
                eng.correct(x, y)
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(a.reps):
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                c = eng.correct(x, y)
                en.record()
                torch.cuda.synchronize()
                assert c == ref, (c, ref)
                best = min(best, st.elapsed_time(en))
            return best

        ec = eng.eng.get_eval_cfg()
        cur = t_eval()
        print(f"chunk {chunk}: default eval cfg {ec[:6]} {cur:.3f} ms", flush=True)
        for op in range(6):
            keep, best_t = ec[op], cur
            for c in cfgs:
                ec[op] = c
                try:
                    eng.eng.set_eval_cfg(ec)
                except RuntimeError:  # eval-only large tiles: conv2-4 forward only
                    continue
                t = t_eval()
                print(f"    op {op} c{c}: {t:.3f} ms", flush=True)
                if t < best_t * 0.99:
                    keep, best_t = c, t
            ec[op] = keep
            eng.eng.set_eval_cfg(ec)
            cur = t_eval()
            print(f"  op {op} -> c{keep}: {cur:.3f} ms", flush=True)
        print(f"chunk {chunk}: EVAL_CFG {','.join(map(str, ec[:6]))} {cur:.3f} ms "
              f"({0.7077e12 / (cur * 1e-3) / 1e12:.1f} TF)", flush=True)
        if best_all is None or cur < best_all[0]:
            best_all = (cur, chunk, list(ec))
        del eng
        torch.cuda.empty_cache()
    print(f"BEST chunk {best_all[1]} eval_cfg {','.join(map(str, best_all[2][:6]))} "
          f"{best_all[0]:.3f} ms")


if __name__ == "__main__":
    main()
