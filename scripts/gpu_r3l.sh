#!/bin/bash
# LDS-DMA for one-wave multi-fragment tiles: kernel tests, eval sweep, driver bench x3
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -v -m gpu \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_l.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/gpu_tests_l.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/eval_sweep.py --chunks 10000 --cfgs 0,3,4,6 > gpurun_out/eval_sweep_l.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/eval_sweep_l.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/ab_combo.sh 3 "X=1" 2>&1 | tee gpurun_out/bench_l.log
