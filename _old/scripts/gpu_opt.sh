#!/bin/bash
# Kernel-optimisation iteration: GPU kernel tests, structure diagnostics, per-op sweep, bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest ${TESTS:-tests/test_hip_kernels.py} -q -m gpu -x > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -z "${SKIP_PEAK:-}" ]; then
  timeout -k 10 120 python scripts/mfma_peak.py > gpurun_out/peak.log 2>&1 || exit $?
  cat gpurun_out/peak.log
fi
timeout -k 10 600 python scripts/op_bench.py --cfgs ${CFGS:-0,1,2,3,4} --splits ${SPLITS:-1,2,4,8,16,32,64} --workers ${WORKERS:-0} --json gpurun_out/op_sweep.json > gpurun_out/op_bench.log 2>&1 || exit $?
grep -E "BEST|best|step" gpurun_out/op_bench.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
