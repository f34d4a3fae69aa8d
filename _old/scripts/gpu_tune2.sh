#!/bin/bash
# tests, per-op sweep (split-K separate/in-launch reduce, stream-K), whole-step tune, bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_hip_kernels.py tests/test_native_runner.py -q -m gpu -x > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-250
timeout -k 10 900 python scripts/op_bench.py --cfgs ${CFGS:-0,3,4,5} --splits ${SPLITS:-1,2,4,8,16,32,64,256,1024} --workers ${WORKERS:-1024,1536,2048,2560,3072,4096} --json gpurun_out/op_sweep.json > gpurun_out/op_bench.log 2>&1 || exit $?
grep -E "BEST|step" gpurun_out/op_bench.log
timeout -k 10 900 python scripts/step_tune.py --sweep gpurun_out/op_sweep.json --top 8 --json gpurun_out/step_tune.json > gpurun_out/step_tune.log 2>&1 || exit $?
tail -6 gpurun_out/step_tune.log
