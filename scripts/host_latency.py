#!/usr/bin/env python3
"""Host/GPU hand-offs at the end of one step, from a rocprofv3 database recorded with
--kernel-trace plus --runtime-trace (HIP API) and/or --marker-trace (roctx ranges).

usage: python scripts/host_latency.py <results.db> [--step N] [--tail US]
Prints, merged in time order and relative to the step's first kernel, the kernels (queue) and
the host regions (thread) of the last TAIL microseconds of step N and the start of step N+1:
which host call issued the apply / the next forward, and how long after the GPU event it
reacted to.
"""
import json
import re
import sqlite3
import subprocess
import sys


def short(name):
    try:
        d = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
    except Exception:
        d = name
    d = re.sub(r"\(.*\)$", "", d).replace("ddl::", "").replace("void ", "")
    return d[:70]


def main():
    db = sys.argv[1]
    step = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else 50
    tail = float(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else 80.0
    c = sqlite3.connect(db)
    ks = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    anchor = "conv1_fwd_kernel"
    starts = [i for i, r in enumerate(ks) if anchor in r[0]]
    i0, i1 = starts[step], starts[step + 1]
    t0, t_next = ks[i0][1], ks[i1][1]
    lo, hi = t_next - tail * 1e3, t_next + 15e3
    ev = []
    for n, s, e, q in ks:
        if e >= lo and s <= hi:
            ev.append((s, e, f"q{q}", short(n) or "(unnamed kernel)"))
    cols = [r[1] for r in c.execute("pragma table_info(regions)")]
    name = next((x for x in ("name", "region_name") if x in cols), None)
    tid = next((x for x in ("tid", "thread_id") if x in cols), None)
    ext = "extdata" if "extdata" in cols else "NULL"
    if name:
        for n, e_, s, e, t in c.execute(
                f"select {name}, {ext}, start, end, {tid or 'NULL'} from regions"):
            if e_:
                try:
                    n = json.loads(e_).get("message", n)
                except ValueError:
                    pass
            if e >= lo and s <= hi:
                ev.append((s, e, f"t{t}", str(n)[:60]))
    ev.sort()
    tids = {}
    for s, e, who, n in ev:
        if who.startswith("t"):
            who = tids.setdefault(who, f"T{len(tids)}")
        print(f"{(s - t0) / 1e3:8.1f} -> {(e - t0) / 1e3:8.1f} ({(e - s) / 1e3:6.1f})  {who:4s} {n}")
    print(f"next step starts at {(t_next - t0) / 1e3:.1f}")


if __name__ == "__main__":
    main()
