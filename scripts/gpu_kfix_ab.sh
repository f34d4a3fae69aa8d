#!/bin/bash
# Window-aware split-K (DDL_KFIX mask + --splits) against the default schedule, same box,
# alternating runs: "name mask splits" triples from the environment (KFIX_CASES, ';'-separated).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
ROUNDS=${ROUNDS:-2}
for i in $(seq $ROUNDS); do
  IFS=';' read -ra CASES <<< "$KFIX_CASES"
  for c in "${CASES[@]}"; do
    read -r name mask spl <<< "$c"
    DDL_KFIX=$mask timeout -k 10 120 python bench.py --tta 0 --steps 400 --warmup 40 --splits $spl > gpurun_out/kf.log 2>&1 || exit $?
    echo "$name $(tail -1 gpurun_out/kf.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
