#!/usr/bin/env python3
"""Per-kernel stall breakdown from rocprofv3 --pmc databases (one or more passes).

usage: python scripts/pmc_summary2.py <pass1.db> [<pass2.db> ...]
Columns (per dispatch, averaged): duration; SQ cycle split active / issue-stall / parked
(disjoint, sum = wave cycles); LDS issue-stall share; MFMA-busy cycles per kernel-cycle per CU;
instruction mix per MFMA; LDS bank-conflict cycles per LDS instruction; TA busy share.
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
    d = re.sub(r"\(.*\)$", "", d).replace("ddl::", "").replace("void ", "")
    return d[:78]


agg = defaultdict(lambda: defaultdict(float))
ndisp = defaultdict(lambda: defaultdict(set))
dur = defaultdict(dict)
for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    for name, disp, cn, val, d in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
        agg[name][cn] += val
        ndisp[name][cn].add((db, disp))
        dur[name][(db, disp)] = d


def per(name, cn):
    n = len(ndisp[name][cn])
    return agg[name][cn] / n if n else float("nan")


print(f"{'kernel':78s} {'us':>6s} {'act%':>5s} {'istl%':>5s} {'park%':>5s} {'lds%':>5s} "
      f"{'mfmaB':>6s} {'valu/m':>6s} {'lds/m':>5s} {'vmem/m':>6s} {'bank/l':>6s} {'ta%':>5s}")
rows = sorted(agg, key=lambda k: -sum(dur[k].values()) / max(1, len(dur[k])) * len(dur[k]))
for name in rows:
    us = sum(dur[name].values()) / len(dur[name]) / 1e3
    wc = per(name, "SQ_WAVE_CYCLES")
    act, ist, park = (100 * per(name, k) / wc for k in
                      ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"))
    lds = 100 * per(name, "SQ_WAIT_INST_LDS") / wc
    gui = per(name, "GRBM_GUI_ACTIVE")  # summed over 8 XCDs
    mf = per(name, "SQ_VALU_MFMA_BUSY_CYCLES")
    mfb = mf / (gui / 8 * 256) if gui == gui and gui else float("nan")  # per CU per cycle
    nm = per(name, "SQ_INSTS_MFMA")
    vm = per(name, "SQ_INSTS_VALU") / nm if nm else float("nan")
    lm = per(name, "SQ_INSTS_LDS") / nm if nm else float("nan")
    mm = per(name, "SQ_INSTS_VMEM_RD") / nm if nm else float("nan")
    bl = per(name, "SQ_LDS_BANK_CONFLICT") / per(name, "SQ_INSTS_LDS") if per(name, "SQ_INSTS_LDS") else 0
    ta = 100 * per(name, "TA_TA_BUSY") / (gui / 8 * 256) if gui == gui and gui else float("nan")
    print(f"{short(name):78s} {us:6.1f} {act:5.1f} {ist:5.1f} {park:5.1f} {lds:5.1f} {mfb:6.2f} "
          f"{vm:6.2f} {lm:5.2f} {mm:6.2f} {bl:6.2f} {ta:5.1f}")
