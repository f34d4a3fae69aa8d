#!/usr/bin/env python3
"""Summarise the roctx ranges of a rocprofv3 --marker-trace database (rocpd sqlite): per range
name, count and mean / total host duration, plus the kernels that started inside one step's
ranges.  usage: python scripts/marker_summary.py <results.db>"""
import json
import sqlite3
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    cand = [t for t in tabs if "region" in t.lower() or "marker" in t.lower()]
    print("tables:", ", ".join(sorted(tabs)))
    rows = []
    for t in cand:
        cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
        name = next((x for x in ("name", "region_name", "message") if x in cols), None)
        if name is None or "start" not in cols or "end" not in cols:
            continue
        ext = "extdata" if "extdata" in cols else "NULL"
        rows = []
        for n, e, s0, s1 in c.execute(f"select {name}, {ext}, start, end from {t}"):
            if e:  # rocprofv3 rocpd: the roctx message is in extdata {"message": ...}
                try:
                    n = json.loads(e).get("message", n)
                except ValueError:
                    pass
            rows.append((n, s0, s1))
        if rows:
            print(f"ranges from {t} ({len(rows)} rows)")
            break
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        if n is None or not str(n).startswith("ddl."):
            continue
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e3
    print(f"{'range':40s} {'count':>7s} {'mean us':>9s} {'total us':>11s}")
    for n, (k, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:40s} {k:7d} {tot / k:9.2f} {tot:11.1f}")


if __name__ == "__main__":
    main()
