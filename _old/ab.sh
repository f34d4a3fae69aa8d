#!/bin/bash
# A/B: pre-session build (_old) vs current tree, same box, alternating
set -u
cd /root/repo
for i in 1 2; do
  (cd _old && timeout -k 10 120 python bench.py --steps 400 --warmup 40 --tta 0 --shard contiguous) | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('OLD', d['ms_per_step'])" || exit 1
  timeout -k 10 120 python bench.py --steps 400 --warmup 40 --tta 0 --shard contiguous | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('NEW-contig', d['ms_per_step'])" || exit 1
  timeout -k 10 120 python bench.py --steps 400 --warmup 40 --tta 0 | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('NEW-flat', d['ms_per_step'])" || exit 1
done
