#!/bin/bash
# xGMI peer exchange on one GPU: multi-process tests (W ranks share the card), native runner
# regression tests, then a short rehearsal bench at W = 2 through torchrun.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_xgmi_gpu.py tests/test_native_runner.py} \
    -x -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/xgmi_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/xgmi_tests.log
exit $rc
