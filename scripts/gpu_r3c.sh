#!/bin/bash
# native-runner tests (incl. the RCCL async self-session rehearsal), bench x3 + kernel-trace
# timeline of the default step, and a roctx marker trace of the native runtime (DDL_TRACE=1)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_native_runner.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_nr.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_nr.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_bench_tl.sh || exit $?
rm -rf gpurun_out/profm
DDL_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace -d $R/gpurun_out/profm -o prof -- python3 bench.py --steps 30 --warmup 5 --prewarm-steps 5 --tta 0 --force-collectives --exchange xgmi > gpurun_out/profm.log 2>&1 || exit $?
python3 scripts/marker_summary.py $(find gpurun_out/profm -name "*.db" | head -n 1) > gpurun_out/marker_summary.txt 2>&1 || exit $?
cat gpurun_out/marker_summary.txt | head -30
