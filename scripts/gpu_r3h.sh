#!/bin/bash
# conv1 weight-gradient direct kernel: kernel tests, A/B, one kernel-trace step timeline
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -v -m gpu \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_h.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests_h.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_combo.sh 2 "DDL_CONV1_WGRAD_DIRECT=0" "DDL_CONV1_WGRAD_DIRECT=1" 2>&1 | tee gpurun_out/ab_h.log
rm -rf gpurun_out/proft
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/proft -o prof -- python3 bench.py --steps 60 --warmup 10 --tta 0 > gpurun_out/proft.log 2>&1 || exit $?
python3 scripts/step_timeline.py $(find gpurun_out/proft -name "*.db" | head -n 1) --step 40 --anchor conv1_fwd_kernel > gpurun_out/timeline_h.txt 2>&1 || exit $?
cat gpurun_out/timeline_h.txt
