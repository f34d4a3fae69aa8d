#!/bin/bash
# eval forward: conv2 on the tap-skipping K map vs the image-major GEMM (full test-set eval time,
# alternating), kernel tests, time to accuracy
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_km.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/gpu_tests_km.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    DDL_EVAL_KMAP2=$v timeout -k 10 120 python scripts/eval_sweep.py --chunks 10000 --cfgs 0 --reps 10 2>/dev/null | grep "default eval" | sed "s/^/KMAP2=$v /"
  done
done 2>&1 | tee gpurun_out/ab_kmap2.log
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/ab_combo.sh 2 "DDL_EVAL_KMAP2=0" "DDL_EVAL_KMAP2=1" 2>&1 | tee -a gpurun_out/ab_kmap2.log
