#!/bin/bash
# Round 4: async gate sweeps the dense DONE words with batched loads: runner suites, benches.

set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 900 python -u -m pytest tests/test_native_runner.py tests/test_xgmi_gpu.py tests/test_gpu_trainer.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread > gpurun_out/r4v_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4v_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4v_tests.log | head; exit $rc; }
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4v_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4v_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4v_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
b local --steps 300 --warmup 20 --tta 0
b forced_xgmi --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
b async_xgmi --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b async_local --mode async --steps 300 --warmup 20 --tta 0
b async_xgmi2 --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b forced_xgmi2 --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
