#!/bin/bash
# rocprofv3 kernel trace of the default bench (N=1) + summary table.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o prof -- python3 bench.py --steps ${STEPS:-100} --warmup 10 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log | cut -c1-200
python3 scripts/prof_summary.py $(find gpurun_out/prof -name "*.db" | head -n 1) --md > gpurun_out/prof_summary.md 2>&1 || exit $?
head -45 gpurun_out/prof_summary.md
