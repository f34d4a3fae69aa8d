#!/bin/bash
# eval-forward tile sweep (10k chunk) on the current build, then one pass of the real-step
# schedule tuner
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/eval_sweep.py --chunks 10000 --cfgs 0,3,6,9,10 > gpurun_out/eval_sweep_r3.log 2>&1
rc=$?; tail -4 gpurun_out/eval_sweep_r3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u scripts/runner_tune.py --passes 1 --steps 400 --json gpurun_out/rtune.json > gpurun_out/rtune.log 2>&1
rc=$?; tail -25 gpurun_out/rtune.log; exit $rc
