#!/usr/bin/env python3
"""Count HIP streams / events created and destroyed per process from rocprofv3 --hip-trace CSV
output (the streams a rank still holds after the bench's release).

usage: python scripts/stream_census.py <dir with *hip_api_trace.csv files>
"""
import csv
import glob
import os
import sys
from collections import Counter, defaultdict

KEEP = ("hipStreamCreate", "hipStreamCreateWithFlags", "hipStreamCreateWithPriority",
        "hipStreamDestroy", "hipEventCreate", "hipEventCreateWithFlags", "hipEventDestroy",
        "hipExtMallocWithFlags", "hipIpcOpenMemHandle", "hipIpcCloseMemHandle",
        "hipHostRegister", "hipHostUnregister")


def main(root):
    per = defaultdict(Counter)
    last = defaultdict(dict)
    files = glob.glob(os.path.join(root, "**", "*hip_api_trace.csv"), recursive=True)
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                fn = row.get("Function") or row.get("Operation") or ""
                pid = row.get("Process_Id") or row.get("Pid") or "?"
                if fn in KEEP:
                    per[pid][fn] += 1
                    last[pid][fn] = int(row.get("End_Timestamp") or 0)
    if not per:
        print(f"no hip API records in {len(files)} file(s) under {root}")
        return 1
    for pid in sorted(per):
        c = per[pid]
        made = sum(v for k, v in c.items() if k.startswith("hipStreamCreate"))
        print(f"pid {pid}: streams created {made} destroyed {c['hipStreamDestroy']} "
              f"(alive at exit {made - c['hipStreamDestroy']}); events created "
              f"{c['hipEventCreate'] + c['hipEventCreateWithFlags']} destroyed "
              f"{c['hipEventDestroy']}; IPC open {c['hipIpcOpenMemHandle']} close "
              f"{c['hipIpcCloseMemHandle']}; uncached allocs {c['hipExtMallocWithFlags']}; "
              f"host register {c['hipHostRegister']} unregister {c['hipHostUnregister']}")
        print("   ", dict(sorted(c.items())))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
