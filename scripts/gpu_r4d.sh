#!/bin/bash
# Round 4: GPU suite on the pruned build (W = 8 one-card, fault injection, MF16), smoke,
# driver bench, async W = 1 over xGMI (AsyncRunner) vs local, MFMA peaks, kernel timelines.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/r4d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4d_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4d_tests.log | head; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4d_smoke.log 2>&1 || { tail gpurun_out/r4d_smoke.log; exit 1; }
tail -1 gpurun_out/r4d_smoke.log
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4d_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4d_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4d_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'])"
}
b driver1 --gpus 1 --steps 20 --warmup 5
b driver2 --gpus 1 --steps 20 --warmup 5
b w300 --steps 300 --warmup 20 --tta 0
b async_xgmi --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
b async_local --mode async --steps 300 --warmup 20 --tta 0
b forced_xgmi --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
b forced_rccl --steps 300 --warmup 20 --tta 0 --force-collectives
timeout -k 10 120 python scripts/mfma_peak.py > gpurun_out/r4d_peak.log 2>&1 || { cat gpurun_out/r4d_peak.log; exit 1; }
head -8 gpurun_out/r4d_peak.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_async
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_async -o prof -- python3 $R/bench.py --mode async --exchange xgmi --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_async.log 2>&1 || exit $?
python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_async -name "*.db" | head -n 1) --step 50 > $R/gpurun_out/timeline_async.txt 2>&1
python3 $R/scripts/marker_summary.py $(find $R/gpurun_out/prof_async -name "*.db" | head -n 1) > $R/gpurun_out/markers_async.txt 2>&1
echo "== async timeline"; cat $R/gpurun_out/timeline_async.txt | tail -40
for v in default "bwd14 x2"; do
  tag=$(echo "$v" | tr -d ' ')
  rm -rf $R/gpurun_out/prof_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$tag -o prof -- python3 $R/scripts/mf16_ab.py --profile "$v" --steps 80 > $R/gpurun_out/prof_$tag.log 2>&1 || exit $?
  python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_$tag -name "*.db" | head -n 1) --step 100 > $R/gpurun_out/timeline_$tag.txt 2>&1 || exit $?
  echo "== $v"; cat $R/gpurun_out/timeline_$tag.txt
done
