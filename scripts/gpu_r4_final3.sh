#!/bin/bash
# Round 4 final GPU tier: full GPU suite, smoke, the driver's bench command (x2), 300-step
# benches (local / async / forced rehearsals), time-to-accuracy, kernel stats of the local step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/r4zz_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4zz_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4zz_tests.log | head; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4zz_smoke.log 2>&1 || { tail gpurun_out/r4zz_smoke.log; exit 1; }
tail -1 gpurun_out/r4zz_smoke.log
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/r4zz_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4zz_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4zz_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
tta = d.get('time_to_acc') or {}
print('$l', d['value'], d['ms_per_step'], d['vs_baseline'], d['config']['exchange'], d['config']['parallelism'], tta.get('time_to_target_s'))"
}
b driver1 --gpus 1 --steps 20 --warmup 5
b driver2 --gpus 1 --steps 20 --warmup 5
b w300 --steps 300 --warmup 20 --tta 0
b w300b --steps 300 --warmup 20 --tta 0
b async_local --mode async --steps 300 --warmup 20 --tta 0
b async_xgmi --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b forced_xgmi --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
b forced_rccl --steps 300 --warmup 20 --tta 0 --force-collectives
b contiguous --steps 300 --warmup 20 --tta 0 --shard contiguous
b tta --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_local
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_local -o prof -- python3 $R/bench.py --steps 100 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_local.log 2>&1 || exit $?
DB=$(find $R/gpurun_out/prof_local -name "*.db" | head -n 1)
python3 $R/scripts/step_timeline.py $DB --step 80 > $R/gpurun_out/timeline_local.txt 2>&1
find $R/gpurun_out/prof_local -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r4zz_kernel_stats.csv \;
rm -rf $R/gpurun_out/prof_local
echo "== local timeline"; cat $R/gpurun_out/timeline_local.txt
