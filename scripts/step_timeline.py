#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 rocpd database (which stream ran what, when).

usage: python scripts/step_timeline.py <results.db> [--step N] [--anchor SUBSTR]
A step starts at each launch of the anchor kernel (default: the conv1 forward kernel, direct
conv1_fwd_kernel or the GEMM ConvFwd<28, 1, 32>).
Prints start offset, duration, gap since the previous kernel end on the same queue, queue id.
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
    d = re.sub(r"\(.*\)$", "", d).replace("ddl::", "").replace("void ", "")
    return d[:80]


def main():
    db = sys.argv[1]
    step = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else 50
    anchor = sys.argv[sys.argv.index("--anchor") + 1] if "--anchor" in sys.argv else None
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    if anchor is None:
        anchor = "conv1_fwd_kernel" if any("conv1_fwd_kernel" in r[0] for r in rows) \
            else "ConvFwd<28, 1, 32>"
    starts = [i for i, r in enumerate(rows) if anchor in r[0]]
    # skip eval launches (huge grids) by requiring the next anchor to be close
    i0, i1 = starts[step], starts[step + 1]
    t0 = rows[i0][1]
    last_end = {}
    busy = 0.0
    spans = []
    for name, s, e, q in rows[i0:i1]:
        gap = (s - last_end[q]) / 1e3 if q in last_end else 0.0
        last_end[q] = e
        spans.append((s, e))
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap{gap:6.1f}  q{q}  {short(name)}")
    spans.sort()
    cur_s, cur_e = spans[0]
    for s, e in spans[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    total = (rows[i1][1] - t0) / 1e3
    print(f"step span {total:.1f} us, GPU busy (any kernel) {busy / 1e3:.1f} us, idle {total - busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
