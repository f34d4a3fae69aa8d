#!/bin/bash
# Kernel-trace timeline of the forced W = 1 xGMI rehearsal (the W > 1 step's structure).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
rm -rf gpurun_out/profx
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profx -o prof -- python3 bench.py --steps 60 --warmup 10 --tta 0 --force-collectives --exchange ${EX:-xgmi} > gpurun_out/profx.log 2>&1 || exit $?
python3 scripts/step_timeline.py $(find gpurun_out/profx -name "*.db" | head -n 1) --step 40 > gpurun_out/timeline_x.txt 2>&1 || exit $?
cat gpurun_out/timeline_x.txt
