#!/bin/bash
# bench (eager default + graph) and a rocprofv3 kernel trace of the default bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-330
timeout -k 10 300 python bench.py --graph ${BENCH_ARGS:-} > gpurun_out/bench_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_graph.log | cut -c1-330
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o prof -- python3 bench.py --steps 100 --warmup 10 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1 || exit $?
python3 scripts/prof_summary.py $(find gpurun_out/prof -name "*.db" | head -n 1) --md > gpurun_out/prof_summary.md 2>&1 || exit $?
python3 scripts/step_timeline.py $(find gpurun_out/prof -name "*.db" | head -n 1) --step 60 > gpurun_out/timeline.txt 2>&1 || exit $?
tail -1 gpurun_out/timeline.txt
