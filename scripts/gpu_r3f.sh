#!/bin/bash
# conv1 direct kernel: kernel tests, then a same-box A/B (step time + time to accuracy)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -v -m gpu \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_f.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_f.log
[ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--steps 400 --warmup 40" bash scripts/ab_combo.sh 3 "DDL_CONV1_DIRECT=0" "DDL_CONV1_DIRECT=1" 2>&1 | tee gpurun_out/ab_f.log
