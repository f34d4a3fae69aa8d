#!/bin/bash
# rocprofv3 kernel trace of the forced 1-rank-collective bench (the W > 1 step structure on
# one GPU) and its per-step timeline.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
rm -rf gpurun_out/prof_forced
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_forced -o prof -- python3 bench.py --steps 100 --warmup 10 --tta 0 --force-collectives ${BENCH_ARGS:-} > gpurun_out/prof_forced.log 2>&1 || exit $?
DB=$(find gpurun_out/prof_forced -name "*.db" | head -n 1)
python3 scripts/prof_summary.py $DB --md > gpurun_out/prof_forced_summary.md 2>&1 || exit $?
python3 scripts/step_timeline.py $DB --step 60 > gpurun_out/timeline_forced.txt 2>&1 || exit $?
cat gpurun_out/timeline_forced.txt
