#!/bin/bash
# kernel tests + driver bench x3 (time to accuracy) + kernel stats of the default bench
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -v -m gpu \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_j.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/gpu_tests_j.log
[ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/ab_combo.sh 3 "X=1" 2>&1 | tee gpurun_out/bench_j.log
rm -rf gpurun_out/profk
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profk -o prof -- python3 bench.py --steps 200 --warmup 20 --tta 0 > gpurun_out/profk.log 2>&1 || exit $?
python3 scripts/prof_summary.py $(find gpurun_out/profk -name "*.db" | head -n 1) --top 30 --md > gpurun_out/r3_kernels_final.md 2>&1 || exit $?
cat gpurun_out/r3_kernels_final.md
