#!/usr/bin/env python3
"""Merged kernel timeline of several processes sharing one GPU (one rocprofv3 database per
rank, same GPU clock): every kernel of every rank in start order over one step window of rank 0.

usage: python scripts/merge_timeline.py <rank0.db> <rank1.db> ... [--step N] [--steps K] [--anchor SUBSTR]
Prints start offset (us, from rank 0's anchor), duration, rank, queue id and the kernel name.
"""
import re
import sqlite3
import subprocess
import sys


def short(name):
    try:
        d = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
    except Exception:
        d = name
    d = d.replace("(anonymous namespace)::", "")
    d = re.sub(r"\(.*\)$", "", d).replace("ddl::", "").replace("void ", "")
    return d[:72] if d else "?"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    opts = sys.argv[1:]
    step = int(opts[opts.index("--step") + 1]) if "--step" in opts else 40
    anchor = opts[opts.index("--anchor") + 1] if "--anchor" in opts else "conv1_fwd_kernel"
    dbs = [a for a in args if a.endswith(".db")]
    rows = []
    for r, db in enumerate(dbs):
        c = sqlite3.connect(db)
        for name, s, e, q in c.execute("select name, start, end, queue_id from kernels"):
            rows.append((s, e, r, q, name))
    rows.sort()
    a0 = [x for x in rows if x[2] == 0 and anchor in x[4]]
    span = int(opts[opts.index("--steps") + 1]) if "--steps" in opts else 2
    t0, t1 = a0[step][0], a0[min(step + span, len(a0) - 1)][0]
    for s, e, r, q, name in rows:
        if e <= t0 or s >= t1:  # (kernels running into the window from before it included)
            continue
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  r{r} q{q:<3} {short(name)}")


if __name__ == "__main__":
    main()
