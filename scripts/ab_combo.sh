#!/bin/bash
# A/B of several environment combinations on the default bench, same box, alternating runs:
#   bash scripts/ab_combo.sh ROUNDS "A=0 B=0" "A=1 B=0" ...
# BENCH_ARGS overrides the bench flags (default: 400 steps, 40 warmup, no time-to-accuracy run);
# with a time-to-accuracy run its seconds are printed too.
set -u
cd "$(dirname "$0")/.."
ROUNDS=$1; shift
ARGS=${BENCH_ARGS:---steps 400 --warmup 40 --tta 0}
for i in $(seq $ROUNDS); do
  for combo in "$@"; do
    env $combo timeout -k 10 150 python bench.py $ARGS 2>/dev/null | python -c "
import sys, json
d = json.loads(sys.stdin.readlines()[-1])
t = d.get('time_to_acc')
print('$combo', d['ms_per_step'], ('tta %.4f s epoch %.4f s' % (t['time_to_target_s'], t['epoch_wall_s'])) if t else '')" || exit 1
  done
done
