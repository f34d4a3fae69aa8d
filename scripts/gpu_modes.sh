#!/bin/bash
# Headline numbers of every mode on one box (README table): the driver's exact command, then
# async W = 1, the forced W > 1 rehearsals (RCCL / xGMI) and the tensor-granular planners.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
out=gpurun_out/modes.log
: > $out
run() {
  echo "== $*" >> $out
  timeout -k 10 240 python bench.py "$@" >> $out 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc ($*)"; tail -5 $out; exit $rc; }
}
run --gpus 1 --steps 20 --warmup 5
for r in 1 2; do
  run --steps 300 --warmup 30 --tta 0
  run --steps 300 --warmup 30 --tta 0 --mode async
  run --steps 300 --warmup 30 --tta 0 --force-collectives
  run --steps 300 --warmup 30 --tta 0 --force-collectives --exchange xgmi
done
run --steps 300 --warmup 30 --tta 0 --shard contiguous
run --steps 300 --warmup 30 --tta 0 --shard greedy
python3 - <<'PY'
import json
cfg = None
for line in open("gpurun_out/modes.log"):
    if line.startswith("=="):
        cfg = line.strip()[3:]
    elif line.startswith("{"):
        r = json.loads(line)
        extra = ""
        if "time_to_target_s" in r:
            extra = f" tta={r['time_to_target_s']}"
        print(f"{cfg:70s} {r['ms_per_step']:.4f} ms  {r['value']:.0f} img/s  "
              f"exchange={r['config'].get('exchange')}{extra}")
PY
