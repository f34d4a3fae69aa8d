#!/usr/bin/env python3
"""Per-stage timing of the fused fc chain launch (csrc/kernels/fc_chain.h) from in-kernel
wall-clock stamps (100 MHz): for each stage, when its items were taken, how long they waited
for their inputs and how long they computed.  usage: python scripts/fc_chain_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddl_amd.models.hip_engine import HipEngine  # noqa: E402
from ddl_amd.models.layout import CANON_OFFSETS, TOTAL_NUMEL  # noqa: E402
from ddl_amd.models.mnist_cnn import init_params_  # noqa: E402

STAGES = [("A fc1 fwd", 128), ("B fc2 fwd", 64), ("C head", 4), ("D fc2 dgrad", 128),
          ("E fc2 wgrad", 66), ("F fc3 wgrad", 65), ("G fc1 dgrad", 128), ("H fc1 wgrad", 160)]


def main():
    dev = torch.device("cuda", 0)
    params = torch.zeros(TOTAL_NUMEL, device=dev)
    init_params_(params, CANON_OFFSETS, 0)
    grads = torch.zeros_like(params)
    eng = HipEngine(params, grads, CANON_OFFSETS, batch=100, graph=False, eval_chunk=100)
    eng.eng.set_fc_chain(True)  # opt-in (api.h)
    x = torch.rand(100, 784, device=dev)
    y = torch.randint(0, 10, (100,), device=dev)
    for i in range(20):
        eng.forward_backward(x, y, 0.5, i)
    n = sum(c for _, c in STAGES)
    st = torch.zeros(n, 8, dtype=torch.int64, device=dev)
    for rep in range(3):
        eng.eng.set_fc_stamps(st)
        eng.forward_backward(x, y, 0.5, 100 + rep)
        torch.cuda.synchronize()
        eng.eng.set_fc_stamps(None)
        s = st.cpu()
        t0 = int(s[:, 0].min())
        print(f"--- run {rep}: launch span {(int(s[:, 2].max()) - t0) / 100:.1f} us "
              f"(first dequeue -> last end), error word {eng.eng.fc_chain_error()}")
        off = 0
        for name, cnt in STAGES:
            r = s[off:off + cnt]
            deq = (r[:, 0] - t0).double() / 100
            ready = torch.where(r[:, 1] > 0, r[:, 1], r[:, 0])
            wait = (ready - r[:, 0]).double() / 100
            comp = (r[:, 2] - ready).double() / 100
            end = (r[:, 2] - t0).double() / 100
            print(f"{name:13s} n={cnt:3d} taken {deq.min():6.1f}-{deq.max():6.1f}  "
                  f"wait med {wait.median():5.1f} max {wait.max():5.1f}  "
                  f"compute med {comp.median():5.1f} max {comp.max():5.1f}  "
                  f"done {end.min():6.1f}-{end.max():6.1f} us")
            if name.startswith("C"):
                for q in range(4):
                    ph = [(int(r[q, j]) - int(r[q, 1])) / 100 for j in (4, 5, 6, 7)]
                    print("    head item %d: staged %.1f, rows done %.1f %.1f %.1f us after ready"
                          % (q, *ph))
            off += cnt


if __name__ == "__main__":
    main()
