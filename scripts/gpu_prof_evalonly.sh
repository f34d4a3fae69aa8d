#!/bin/bash
# kernel stats of the full test-set eval forward alone (eval_sweep's timing loop)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
rm -rf gpurun_out/profev
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profev -o prof -- python3 scripts/eval_sweep.py --chunks 10000 --cfgs 0 --reps 5 > gpurun_out/profev.log 2>&1 || exit $?
python3 scripts/prof_summary.py $(find gpurun_out/profev -name "*.db" | head -n 1) --top 20 --md > gpurun_out/r3_eval_kernels.md 2>&1 || exit $?
cat gpurun_out/r3_eval_kernels.md
