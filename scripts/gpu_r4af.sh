#!/bin/bash
# Round 4: memory-side PMC pass on the default step (L2 hit rate per kernel) for next round's
# forward / backward GEMM work.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc3
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc3 -o pmc -- python3 $R/scripts/pmc_probe.py > $R/gpurun_out/pmc3.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 $R/gpurun_out/pmc3.log
[ $rc -ne 0 ] && exit $rc
DB=$(find $R/gpurun_out/pmc3 -name "*.db" | head -n 1)
python3 - "$DB" > $R/gpurun_out/pmc3_summary.txt <<'PY'
import re, sqlite3, subprocess, sys
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
agg = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(set)
q = None
for t in ("counters_collection", "pmc_events"):
    if t in tabs:
        cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
        print(t, cols[:20])
rows = c.execute("select * from counters_collection limit 1").fetchall() if "counters_collection" in tabs else []
print(rows[:1])
PY
cat $R/gpurun_out/pmc3_summary.txt | head -20
