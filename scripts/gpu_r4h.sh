#!/bin/bash
# Round 4: async board + device-resident table (small kernargs).
# Async GPU tests, benches (async xGMI W=1 vs local), traced timeline with host markers.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "async" > gpurun_out/r4h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4h_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4h_tests.log | head; exit $rc; }
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4h_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4h_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4h_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
b async_xgmi --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b async_local --mode async --steps 300 --warmup 20 --tta 0
b async_xgmi2 --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b async_xgmi_none --mode async --exchange xgmi --shard none --steps 300 --warmup 20 --tta 0
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_async
export DDL_TRACE=1
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_async -o prof -- python3 $R/bench.py --mode async --exchange xgmi --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_async.log 2>&1 || exit $?
unset DDL_TRACE
python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_async -name "*.db" | head -n 1) --step 50 > $R/gpurun_out/timeline_async.txt 2>&1
python3 $R/scripts/marker_summary.py $(find $R/gpurun_out/prof_async -name "*.db" | head -n 1) > $R/gpurun_out/markers_async.txt 2>&1
echo "== async timeline"; tail -45 $R/gpurun_out/timeline_async.txt
echo "== markers"; head -40 $R/gpurun_out/markers_async.txt
