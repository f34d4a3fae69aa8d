#!/bin/bash
# The driver's exact bench command next to longer windows, alternating, on one box:
# explains a gap between the 20-step driver number and the 200-step numbers.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
out=gpurun_out/driver_bench.log
: > $out
for r in 1 2 3; do
  for cfg in "--steps 20 --warmup 5" "--steps 200 --warmup 20" ${EXTRA_CFG:+"$EXTRA_CFG"}; do
    echo "== round $r: $cfg" >> $out
    timeout -k 10 200 python bench.py --gpus 1 $cfg --tta 0 >> $out 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc ($cfg)"; tail -5 $out; exit $rc; }
  done
done
python - <<'EOF'
import json
cfg = None
for line in open("gpurun_out/driver_bench.log"):
    if line.startswith("=="):
        cfg = line.strip()
    elif line.startswith("{"):
        r = json.loads(line)
        print(cfg, r["ms_per_step"], r["value"])
EOF
