#!/bin/bash
# A/B of several environment combinations on the default bench, same box, alternating runs:
#   bash scripts/ab_combo.sh ROUNDS "A=0 B=0" "A=1 B=0" ...
set -u
cd "$(dirname "$0")/.."
ROUNDS=$1; shift
for i in $(seq $ROUNDS); do
  for combo in "$@"; do
    env $combo timeout -k 10 120 python bench.py --steps 400 --warmup 40 --tta 0 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('$combo', d['ms_per_step'])" || exit 1
  done
done
