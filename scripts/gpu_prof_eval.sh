#!/bin/bash
# Kernel stats of the time-to-accuracy epoch (500 steps + 50 full test-set evals): where the
# eval forward spends its time.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
rm -rf gpurun_out/profe
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profe -o prof -- python3 bench.py --steps 20 --warmup 5 --prewarm-steps 0 > gpurun_out/profe.log 2>&1 || exit $?
tail -1 gpurun_out/profe.log | cut -c1-200
python3 scripts/prof_summary.py $(find gpurun_out/profe -name "*.db" | head -n 1) --top 40 > gpurun_out/prof_eval_summary.txt 2>&1 || exit $?
cat gpurun_out/prof_eval_summary.txt
