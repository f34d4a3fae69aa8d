#!/bin/bash
# Round 4: sync W>1 READY flags on every segment (default mode 2): tests, A/B, benches, timeline.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 700 python -u -m pytest tests/test_native_runner.py tests/test_xgmi_gpu.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "not async or resume" > gpurun_out/r4o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4o_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4o_tests.log | head; exit $rc; }
timeout -k 10 300 python scripts/ready_ab.py > gpurun_out/r4o_ready_ab.log 2>&1 || { tail -20 gpurun_out/r4o_ready_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4o_ready_ab.log
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4o_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4o_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4o_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
b forced_xgmi --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
b forced_rccl --steps 300 --warmup 20 --tta 0 --force-collectives
b local --steps 300 --warmup 20 --tta 0
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_forced_xgmi
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_forced_xgmi -o prof -- python3 $R/bench.py --force-collectives --exchange xgmi --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_forced_xgmi.log 2>&1 || exit $?
python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_forced_xgmi -name "*.db" | head -n 1) --step 50 > $R/gpurun_out/timeline_forced_xgmi.txt 2>&1
echo "== forced xgmi"; tail -30 $R/gpurun_out/timeline_forced_xgmi.txt
