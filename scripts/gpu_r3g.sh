#!/bin/bash
# conv1 weight-gradient direct kernel: kernel + runner tests, then a same-box A/B
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_native_runner.py -x -v -m gpu \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_g.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_g.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_combo.sh 3 "DDL_CONV1_WGRAD_DIRECT=0" "DDL_CONV1_WGRAD_DIRECT=1" 2>&1 | tee gpurun_out/ab_g.log
