#!/bin/bash
# One build->measure iteration on the GPU box: kernel tests, bench, rocprofv3 kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_hip_kernels.py} -q -m gpu > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 20 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o prof -- python3 bench.py --steps 50 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
