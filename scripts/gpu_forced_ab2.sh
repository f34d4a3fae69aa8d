#!/bin/bash
# native-runner tests, then forced W > 1 rehearsals (RCCL / xGMI) with the segment event bound
# to the last launch (default) vs a marker record (DDL_EXT_EVENT=0), alternating; a timeline.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_native_runner.py -x -q -m gpu -p no:cacheprovider \
    --timeout 200 --timeout-method thread > gpurun_out/t_nr.log 2>&1
rc=$?; tail -1 gpurun_out/t_nr.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for ex in rccl xgmi; do
    for ee in 1 0; do
      DDL_EXT_EVENT=$ee timeout -k 10 200 python bench.py --steps 300 --warmup 30 --tta 0 --force-collectives --exchange $ex > gpurun_out/fab.log 2>&1 || { tail -5 gpurun_out/fab.log; exit 1; }
      echo "$ex ext=$ee $(tail -1 gpurun_out/fab.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
bash scripts/gpu_prof_forced.sh
