#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -v -m gpu -k "odd_batches or conv1" \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_m.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/gpu_tests_m.log | head -20; exit $rc
