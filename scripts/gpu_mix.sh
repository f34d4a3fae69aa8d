#!/bin/bash
# dual launches: proportional interleave of the two problems' blocks per layer (DDL_DUAL_MIX)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu -k "backward_modes or conv1_wgrad or split_k" \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_mix.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/gpu_tests_mix.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_combo.sh 3 "DDL_DUAL_MIX=0" "DDL_DUAL_MIX=1024" "DDL_DUAL_MIX=4096" "DDL_DUAL_MIX=16384" "DDL_DUAL_MIX=21504" 2>&1 | tee gpurun_out/ab_mix.log
