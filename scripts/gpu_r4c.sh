#!/bin/bash
# Round 4: the pruned build on one box — GPU suite (incl. W = 8 one-card and fault injection),
# smoke, driver bench, MFMA peaks, MF16 timeline.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|SKIPPED|ERROR" gpurun_out/r4c_tests.log | tail -5; tail -3 gpurun_out/r4c_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c_smoke.log 2>&1 || { tail gpurun_out/r4c_smoke.log; exit 1; }
tail -1 gpurun_out/r4c_smoke.log
for k in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4c_bench$k.log 2>&1 || { tail gpurun_out/r4c_bench$k.log; exit 1; }
  tail -1 gpurun_out/r4c_bench$k.log | cut -c1-240
done
timeout -k 10 120 python scripts/mfma_peak.py > gpurun_out/r4c_peak.log 2>&1 || { cat gpurun_out/r4c_peak.log; exit 1; }
head -8 gpurun_out/r4c_peak.log
cd /tmp && export TMPDIR=/tmp
for v in default "bwd14 x2"; do
  tag=$(echo "$v" | tr -d ' ')
  rm -rf $R/gpurun_out/prof_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$tag -o prof -- python3 $R/scripts/mf16_ab.py --profile "$v" --steps 80 > $R/gpurun_out/prof_$tag.log 2>&1 || exit $?
  python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_$tag -name "*.db" | head -n 1) --step 100 > $R/gpurun_out/timeline_$tag.txt 2>&1 || exit $?
  echo "== $v"; cat $R/gpurun_out/timeline_$tag.txt
done
