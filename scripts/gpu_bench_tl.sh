#!/bin/bash
# bench x3 + one kernel-trace timeline of the default step
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
for k in 1 2 3; do
  timeout -k 10 120 python bench.py --tta 0 --steps 300 ${BENCH_ARGS:-} > gpurun_out/btl.log 2>&1 || exit $?
  echo "run $k $(tail -1 gpurun_out/btl.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
rm -rf gpurun_out/proft
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/proft -o prof -- python3 bench.py --steps 60 --warmup 10 --tta 0 ${BENCH_ARGS:-} > gpurun_out/proft.log 2>&1 || exit $?
python3 scripts/step_timeline.py $(find gpurun_out/proft -name "*.db" | head -n 1) --step 40 > gpurun_out/timeline_t.txt 2>&1 || exit $?
cat gpurun_out/timeline_t.txt
