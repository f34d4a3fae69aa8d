#!/bin/bash
# Round 4: real-step tune of the forward convolutions including the multi-wave tile configs.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u scripts/runner_tune.py --passes 1 --steps 400 --gain 0.002 --multiwave --ops 1,2,3,4,5 --json gpurun_out/r4ad_tune.json > gpurun_out/r4ad_tune.log 2>&1 || { tail -20 gpurun_out/r4ad_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4ad_tune.log
