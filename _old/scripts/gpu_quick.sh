#!/bin/bash
# tests + bench (graph on/off) + op timing of a few ops
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest ${TESTS:-tests/test_hip_kernels.py} -q -m gpu > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-260
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-graph > gpurun_out/bench_ng.log 2>&1 || exit $?
tail -1 gpurun_out/bench_ng.log | cut -c1-260
