#!/bin/bash
# Round 4: xGMI owner kernel stores this rank's own parameter copy at device scope (sc1):
# forced xGMI benches + timeline (does the next forward recover its local-step speed?).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_native_runner.py tests/test_xgmi_gpu.py -x -q -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "not async" > gpurun_out/r4ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4ab_tests.log
[ $rc -ne 0 ] && exit $rc
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4ab_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4ab_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4ab_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
b local --steps 300 --warmup 20 --tta 0
b forced_xgmi --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
b forced_xgmi2 --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_fx
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_fx -o prof -- python3 $R/bench.py --force-collectives --exchange xgmi --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_fx.log 2>&1 || exit $?
python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_fx -name "*.db" | head -n 1) --step 50 > $R/gpurun_out/timeline_forced_xgmi.txt 2>&1
rm -rf $R/gpurun_out/prof_fx
echo "== forced xgmi"; cat $R/gpurun_out/timeline_forced_xgmi.txt
