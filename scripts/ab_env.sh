#!/bin/bash
# A/B of one environment knob on the default bench, same box, alternating runs:
#   bash scripts/ab_env.sh VAR "val1 val2 ..." [rounds]
set -u
cd "$(dirname "$0")/.."
VAR=$1; VALS=$2; ROUNDS=${3:-2}
for i in $(seq $ROUNDS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 120 python bench.py --steps 400 --warmup 40 --tta 0 | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('$VAR=$v', d['ms_per_step'])" || exit 1
  done
done
