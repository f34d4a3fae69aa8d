#!/bin/bash
# last-segment Adam fused into the conv1 weight-gradient launch: tests, A/B, timeline (knob on)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_native_runner.py -x -v -m gpu \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_i.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests_i.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_combo.sh 2 "DDL_FINAL_IN_REDUCE=0" "DDL_FINAL_IN_REDUCE=1" 2>&1 | tee gpurun_out/ab_i.log
rm -rf gpurun_out/proft
DDL_FINAL_IN_REDUCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/proft -o prof -- python3 bench.py --steps 60 --warmup 10 --tta 0 > gpurun_out/proft.log 2>&1 || exit $?
python3 scripts/step_timeline.py $(find gpurun_out/proft -name "*.db" | head -n 1) --step 40 --anchor conv1_fwd_kernel > gpurun_out/timeline_i.txt 2>&1 || exit $?
cat gpurun_out/timeline_i.txt
