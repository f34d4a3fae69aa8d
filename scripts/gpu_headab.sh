#!/bin/bash
# A/B of the fused fc2-reduce + head kernel: bench pairs and one kernel-trace timeline each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
for k in 1 2; do
  for f in 0 1; do
    DDL_FUSE_HEAD=$f timeout -k 10 120 python bench.py --tta 0 --steps 300 > gpurun_out/hab_$f.log 2>&1 || exit $?
    echo "fuse=$f $(tail -1 gpurun_out/hab_$f.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
for f in 0 1; do
  rm -rf gpurun_out/prof$f
  DDL_FUSE_HEAD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof$f -o prof -- python3 bench.py --steps 60 --warmup 10 --tta 0 > gpurun_out/prof$f.log 2>&1 || exit $?
  python3 scripts/step_timeline.py $(find gpurun_out/prof$f -name "*.db" | head -n 1) --step 40 > gpurun_out/timeline$f.txt 2>&1 || exit $?
  grep -iE "head|FcFwd|span" gpurun_out/timeline$f.txt
done
