#!/bin/bash
# Baseline (stock torch) bench, no-graph bench, and a rocprofv3 kernel-trace profile.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --engine torch > gpurun_out/bench_torch.log 2>&1 || exit $?
tail -1 gpurun_out/bench_torch.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-graph > gpurun_out/bench_nograph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_nograph.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o prof -- python3 bench.py --steps 50 --warmup 5 > gpurun_out/prof.log 2>&1 || exit $?
find gpurun_out/prof -name "*stats*" | head
