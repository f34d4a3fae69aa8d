#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd sqlite database: per-kernel count / total / mean / share.

usage: python scripts/prof_summary.py <results.db> [--top N] [--md]
"""
import re
import sqlite3
import subprocess
import sys
from collections import defaultdict


def short(name: str) -> str:
    try:
        d = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
    except Exception:
        d = name
    d = re.sub(r"\(.*\)$", "", d)
    d = d.replace("ddl::", "")
    return d[:110]


def main():
    db = sys.argv[1]
    top = 60
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    namecol = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {namecol}, start, end from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    t_min, t_max = None, None
    for n, s, e in rows:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
        t_min = s if t_min is None else min(t_min, s)
        t_max = e if t_max is None else max(t_max, e)
    tot = sum(v[1] for v in agg.values())
    md = "--md" in sys.argv
    if md:
        print("| kernel | calls | total us | mean us | % |\n|---|---|---|---|---|")
    for n, (cnt, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        s = short(n)
        if md:
            print(f"| `{s}` | {cnt} | {us:.1f} | {us / cnt:.2f} | {100 * us / tot:.1f} |")
        else:
            print(f"{cnt:7d} {us:12.1f} us {us / cnt:9.2f} us {100 * us / tot:5.1f}%  {s}")
    print(f"\nkernel time total {tot:.1f} us over {len(rows)} dispatches; "
          f"trace span {(t_max - t_min) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
