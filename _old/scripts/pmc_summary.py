#!/usr/bin/env python3
"""Per-kernel PMC summary from a rocprofv3 --pmc database (rocpd sqlite).
usage: python scripts/pmc_summary.py <pmc_results.db>"""
import re
import sqlite3
import subprocess
import sys
from collections import defaultdict


def short(n):
    try:
        d = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip() or n
    except Exception:
        d = n
    return re.sub(r"\(.*\)$", "", d).replace("ddl::", "")[:90]


c = sqlite3.connect(sys.argv[1])
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
dur = defaultdict(dict)
for name, disp, cn, val, d, vg, ag in c.execute(
        "select kernel_name, dispatch_id, counter_name, value, duration, vgpr_count, accum_vgpr_count from counters_collection"):
    agg[name][cn] += val
    cnt[name].add(disp)
    dur[name][disp] = d
    agg[name]["_vgpr"] = vg
    agg[name]["_agpr"] = ag
print(f"{'kernel':90s} {'n':>3s} {'us':>7s} {'MFMAbusy%':>9s} {'waitLDS%':>8s} {'waitAny%':>8s} {'bankcf':>8s} {'waves':>7s} {'v/a':>7s}")
for name, d in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]].values())):
    n = len(cnt[name])
    us = sum(dur[name].values()) / n / 1e3
    busy = d.get("SQ_BUSY_CU_CYCLES", 0) * 4  # quad-cycles per CU aggregated
    mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    wc = d.get("SQ_WAVE_CYCLES", 0)
    mfp = 100 * mf / (busy * 4) if busy else 0  # 4 SIMDs per CU
    wl = 100 * d.get("SQ_WAIT_INST_LDS", 0) / wc if wc else 0
    wa = 100 * d.get("SQ_WAIT_ANY", 0) / wc if wc else 0
    print(f"{short(name):90s} {n:3d} {us:7.1f} {mfp:9.1f} {wl:8.1f} {wa:8.1f} {d.get('SQ_LDS_BANK_CONFLICT', 0) / n:8.0f} {d.get('SQ_WAVES', 0) / n:7.0f} {int(d['_vgpr'])}/{int(d['_agpr'])}")
