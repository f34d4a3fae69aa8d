#!/bin/bash
# kernel numerics tests, then bench x3 + one kernel-trace timeline of the default step
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_hip_kernels.py tests/test_native_runner.py} \
    -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/kb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/kb_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_bench_tl.sh
