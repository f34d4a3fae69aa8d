#!/bin/bash
# Round 4: CFG_MF16 numerics + real-step A/B against the default schedule, one box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v -k "mf16 or gradients_match or backward_modes" \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/r4a_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/mf16_ab.py --steps 300 --rounds 3 --scales 1,2 > gpurun_out/r4a_ab.log 2>&1
rc=$?; cat gpurun_out/r4a_ab.log | tail -12
exit $rc
