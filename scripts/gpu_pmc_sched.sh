#!/bin/bash
# PMC (VALU / SALU / MFMA instruction counts) of one op under several schedules.
set -u
cd "$(dirname "$0")/.."
R=$PWD
cd /tmp && export TMPDIR=/tmp
OP=${OP:-conv3_dgrad}
i=0
for sched in "--splits 1" "--splits 8" "--splits 8 --inline" "--workers 2048" "--splits 16"; do
  i=$((i+1))
  rm -rf $R/gpurun_out/pmcs$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $R/gpurun_out/pmcs$i -o p -- python3 $R/scripts/pmc_sched_probe.py --op $OP $sched > $R/gpurun_out/pmcs$i.log 2>&1 || exit 1
  python3 - "$R/gpurun_out/pmcs$i" "$sched" <<'PY'
import glob, sqlite3, sys
from collections import defaultdict
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
agg = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for name, disp, cn, val in c.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection"):
    if "gemm" not in name and "reduce" not in name: continue
    k = name.split("<")[0].split()[-1]
    agg[k][cn] += val; n[k].add(disp)
for k, d in agg.items():
    m = d["SQ_INSTS_MFMA"] or 1
    print(f"{sys.argv[2]:22s} {k:22s} disp {len(n[k]):3d} waves/disp {d['SQ_WAVES']/len(n[k]):8.0f} "
          f"mfma/disp {d['SQ_INSTS_MFMA']/len(n[k]):9.0f} valu/m {d['SQ_INSTS_VALU']/m:5.2f} "
          f"salu/m {d['SQ_INSTS_SALU']/m:5.2f} smem/m {d['SQ_INSTS_SMEM']/m:5.2f} lds/m {d['SQ_INSTS_LDS']/m:5.2f} "
          f"vmrd/m {d['SQ_INSTS_VMEM_RD']/m:5.2f} vmwr/m {d['SQ_INSTS_VMEM_WR']/m:5.2f}")
PY
done
