#!/bin/bash
# Round 4: async runner yields the HIP runtime to the local PS service after the last push.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_gpu_trainer.py tests/test_native_runner.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "async or push_tails or resume" > gpurun_out/r4r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4r_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4r_tests.log | head; exit $rc; }
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4r_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4r_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4r_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
b async_xgmi --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b async_local --mode async --steps 300 --warmup 20 --tta 0
b async_xgmi2 --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b async_local2 --mode async --steps 300 --warmup 20 --tta 0
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_async_rt
export DDL_TRACE=1
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace -d $R/gpurun_out/prof_async_rt -o prof -- python3 $R/bench.py --mode async --exchange xgmi --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_async_rt.log 2>&1 || exit $?
unset DDL_TRACE
DB=$(find $R/gpurun_out/prof_async_rt -name "*.db" | head -n 1)
python3 $R/scripts/host_latency.py $DB --step 50 --tail 70 > $R/gpurun_out/latency_async.txt 2>&1
rm -rf $R/gpurun_out/prof_async_rt
echo "== latency"; cat $R/gpurun_out/latency_async.txt | head -60
