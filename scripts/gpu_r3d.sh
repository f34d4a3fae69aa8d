#!/bin/bash
# GPU tier + same-box A/B of the last segment's update inside conv1's reduce launch.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_driver.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_env.sh DDL_FINAL_IN_REDUCE "0 1" 3 2>&1 | tee gpurun_out/ab_final.log
