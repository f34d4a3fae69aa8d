#!/bin/bash
# GPU suite + driver bench x3 (time to accuracy) + 300-step windows after the re-tune
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/gpu_tests_k.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/gpu_tests_k.log)"
[ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/ab_combo.sh 3 "X=1" 2>&1 | tee gpurun_out/bench_k.log
BENCH_ARGS="--steps 300 --warmup 20 --tta 0" bash scripts/ab_combo.sh 2 "X=1" 2>&1 | tee -a gpurun_out/bench_k.log
