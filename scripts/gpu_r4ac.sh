#!/bin/bash
# Round 4: READY-flag modes and the high-priority-stream fallback, bit-identical (GPU test).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_native_runner.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "ready_flag or forced" > gpurun_out/r4ac_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r4ac_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r4ac_tests.log | head -20; exit $rc; }
exit 0
