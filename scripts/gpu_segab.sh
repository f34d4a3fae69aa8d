#!/bin/bash
# A/B of the bucket issue points in the forced W = 1 rehearsals (xGMI and RCCL), alternating.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for k in 1 2; do
  for ex in xgmi rccl; do
    for m in ${MAPS:-"0,1,2,3" "1,1,2,3" "1,1,3,3"}; do
      DDL_SEG_ISSUE=$m timeout -k 10 120 python bench.py --tta 0 --steps 300 --force-collectives --exchange $ex > gpurun_out/segab.log 2>&1 || exit $?
      echo "$ex $m $(tail -1 gpurun_out/segab.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
