#!/bin/bash
# forced xGMI rehearsal: workgroups per bucket kernel (DDL_XGMI_SLICES), alternating
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for r in 1 2; do
  for s in ${SLICES:-128 64 32 16}; do
    DDL_XGMI_SLICES=$s timeout -k 10 200 python bench.py --steps 300 --warmup 30 --tta 0 --force-collectives --exchange xgmi > gpurun_out/xs.log 2>&1 || { tail -5 gpurun_out/xs.log; exit 1; }
    echo "slices=$s $(tail -1 gpurun_out/xs.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
