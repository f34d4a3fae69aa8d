#!/bin/bash
# GPU validation: kernel numerics tests, smoke, short bench.  Stops at the first fault.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_hip_kernels.py} -q -m gpu -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
