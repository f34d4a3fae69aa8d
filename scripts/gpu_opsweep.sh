#!/bin/bash
# per-op split / stream-K sweep of the conv forward GEMMs on several in-tree builds (DDL_SO)
#   SOS="_C.so _C_off.so" OPS=conv2_fwd,conv3_fwd,conv4_fwd bash scripts/gpu_opsweep.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for so in ${SOS:-_C.so}; do
  echo "== $so"
  DDL_SO=$so timeout -k 10 300 python scripts/op_bench.py --ops ${OPS:-conv2_fwd,conv3_fwd,conv4_fwd} \
      --cfgs ${CFGS:-3} --splits ${SPLITS:-1,2,3,4,6,8,12,16} --workers ${WORKERS:-0,1024,2048,3072,4096} \
      --iters 100 --no-step > gpurun_out/opsweep_$so.log 2>&1 || { tail -5 gpurun_out/opsweep_$so.log; exit 1; }
  grep -v "^BEST" gpurun_out/opsweep_$so.log
done
