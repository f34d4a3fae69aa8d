#!/bin/bash
# Forced 1-rank rehearsal of the W > 1 step (bench.py --force-collectives): an env knob A/B,
# alternating runs on one box.  usage: KNOB=DDL_EXT_EVENT A=1 B=0 bash scripts/gpu_forced_ab.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
KNOB=${KNOB:-DDL_EXT_EVENT}; A=${A:-1}; B=${B:-0}
out=gpurun_out/forced_ab.log
: > $out
for r in 1 2 3; do
  for ex in ${EXCHANGES:-xgmi rccl}; do
    for v in $A $B; do
      echo "== $KNOB=$v exchange=$ex" >> $out
      env $KNOB=$v timeout -k 10 120 python bench.py --force-collectives --exchange $ex \
          --steps ${STEPS:-200} --tta 0 >> $out 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc ($KNOB=$v $ex)"; tail -5 $out; exit $rc; }
    done
  done
done
python - <<'EOF'
import json, collections
res = collections.defaultdict(list)
cfg = None
for line in open("gpurun_out/forced_ab.log"):
    if line.startswith("=="):
        cfg = line[3:].strip()
    elif line.startswith("{"):
        res[cfg].append(json.loads(line)["ms_per_step"])
for k, v in res.items():
    print(f"{k}: {v}")
EOF
