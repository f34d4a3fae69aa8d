#!/bin/bash
# Round 4: async benches after caching the gate's stream-priority check (x3, alternating with local).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_xgmi_gpu.py -x -q -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "async or push_tails" > gpurun_out/r4aa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4aa_tests.log
[ $rc -ne 0 ] && exit $rc
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4aa_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4aa_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4aa_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
for i in 1 2 3; do
  b async_xgmi$i --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
  b local$i --steps 300 --warmup 20 --tta 0
done
