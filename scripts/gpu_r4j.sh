#!/bin/bash
# Round 4: async W=1 parity probe (xGMI native / Python vs local), async benches, forced timelines.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 300 python scripts/async_parity_probe.py > gpurun_out/r4j_probe.log 2>&1 || { tail -20 gpurun_out/r4j_probe.log; exit 1; }
cat gpurun_out/r4j_probe.log | grep -v amdgpu.ids
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4j_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4j_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4j_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
b async_xgmi --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b async_local --mode async --steps 300 --warmup 20 --tta 0
b async_xgmi2 --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_async
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_async -o prof -- python3 $R/bench.py --mode async --exchange xgmi --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_async.log 2>&1 || exit $?
python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_async -name "*.db" | head -n 1) --step 50 > $R/gpurun_out/timeline_async.txt 2>&1
echo "== async timeline"; tail -30 $R/gpurun_out/timeline_async.txt
for v in xgmi rccl; do
  rm -rf $R/gpurun_out/prof_forced_$v
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_forced_$v -o prof -- python3 $R/bench.py --force-collectives --exchange $v --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_forced_$v.log 2>&1 || exit $?
  python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_forced_$v -name "*.db" | head -n 1) --step 50 > $R/gpurun_out/timeline_forced_$v.txt 2>&1
  echo "== forced $v"; tail -30 $R/gpurun_out/timeline_forced_$v.txt
done
