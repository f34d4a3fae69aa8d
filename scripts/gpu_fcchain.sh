#!/bin/bash
# fused fc chain: kernel numerics, an alternating A/B against the six launches, a timeline
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_hk.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_hk.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/gpu_tests_hk.log | head; exit $rc; }
for r in 1 2 3; do
  for v in 1 0; do
    DDL_FC_CHAIN=$v timeout -k 10 120 python bench.py --tta 0 --steps 300 > gpurun_out/fcab.log 2>&1 || { tail -5 gpurun_out/fcab.log; exit 1; }
    echo "DDL_FC_CHAIN=$v $(tail -1 gpurun_out/fcab.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
timeout -k 10 120 python scripts/fc_chain_probe.py || exit $?
rm -rf gpurun_out/proft
DDL_FC_CHAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/proft -o prof -- python3 bench.py --steps 60 --warmup 10 --tta 0 > gpurun_out/proft.log 2>&1 || exit $?
python3 scripts/step_timeline.py $(find gpurun_out/proft -name "*.db" | head -n 1) --step 40 > gpurun_out/timeline_t.txt 2>&1 || exit $?
cat gpurun_out/timeline_t.txt
