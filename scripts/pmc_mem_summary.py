#!/usr/bin/env python3
"""Per-kernel memory-hierarchy counters from one rocprofv3 --pmc pass (scripts/gpu.sh pmc):
vector L1 (TCP) accesses / L2 requests / stall cycles, L2 (TCC) hit rate, TA and TD busy share.

usage: python scripts/pmc_mem_summary.py <pass.db>
"""
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
    return re.sub(r"\(.*\)$", "", d).replace("ddl::", "").replace("void ", "")[:74]


agg = defaultdict(lambda: defaultdict(float))
nd = defaultdict(lambda: defaultdict(set))
dur = defaultdict(dict)
c = sqlite3.connect(sys.argv[1])
for name, disp, cn, val, d in c.execute(
        "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
    agg[name][cn] += val
    nd[name][cn].add(disp)
    dur[name][disp] = d


def per(name, cn):
    if not nd[name][cn] and nd[name][cn + "_sum"]:
        cn += "_sum"  # rocprofv3 stores the XCD-summed forms under their _sum names
    n = len(nd[name][cn])
    return agg[name][cn] / n if n else float("nan")


print(f"{'kernel':74s} {'us':>6s} {'L1acc/cyc':>9s} {'L2req/cyc':>9s} {'L2hit%':>6s} "
      f"{'tcpStl%':>7s} {'pend%':>6s} {'ta%':>5s} {'td%':>5s} {'L2rdreq':>9s} {'vmemrd':>8s}")
rows = sorted(agg, key=lambda k: -sum(dur[k].values()))
for name in rows:
    us = sum(dur[name].values()) / len(dur[name]) / 1e3
    gui = per(name, "GRBM_GUI_ACTIVE")
    cu_cyc = gui / 8 * 256 if gui == gui and gui else float("nan")  # CU-cycles of the kernel
    acc = per(name, "TCP_TOTAL_CACHE_ACCESSES") / cu_cyc
    req = per(name, "TCP_TCC_READ_REQ") / cu_cyc
    hit, miss = per(name, "TCC_HIT"), per(name, "TCC_MISS")
    hr = 100 * hit / (hit + miss) if hit + miss else float("nan")
    stl = 100 * per(name, "TCP_TCR_TCP_STALL_CYCLES") / cu_cyc
    pend = 100 * per(name, "TCP_PENDING_STALL_CYCLES") / cu_cyc
    ta = 100 * per(name, "TA_TA_BUSY") / cu_cyc
    td = 100 * per(name, "TD_TD_BUSY") / cu_cyc
    print(f"{short(name):74s} {us:6.1f} {acc:9.3f} {req:9.3f} {hr:6.1f} {stl:7.2f} {pend:6.2f} "
          f"{ta:5.1f} {td:5.1f} {per(name, 'TCP_TCC_READ_REQ'):9.0f} "
          f"{per(name, 'SQ_INSTS_VMEM_RD'):8.0f}")
