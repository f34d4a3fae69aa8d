#!/bin/bash
# Stock-PyTorch faithful baseline + HIP bench + rocprofv3 kernel trace of the HIP bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --engine torch > gpurun_out/bench_torch.log 2>&1 || exit $?
tail -1 gpurun_out/bench_torch.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-200
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o prof -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/prof.log 2>&1 || exit $?
rm -rf gpurun_out/prof_torch
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_torch -o prof -- python3 bench.py --steps 100 --warmup 10 --engine torch > gpurun_out/prof_torch.log 2>&1 || exit $?
echo done
