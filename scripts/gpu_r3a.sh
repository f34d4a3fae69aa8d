#!/bin/bash
# round 3 first validation: GPU tests (one process), then the forced-rehearsal event A/B
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_forced_ab.sh
