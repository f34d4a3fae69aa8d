#!/bin/bash
# Round 4: real-step schedule re-tune on the current build (incl. CFG_MF16 candidates).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u scripts/runner_tune.py --passes 2 --steps 400 --gain 0.002 --json gpurun_out/r4u_tune.json > gpurun_out/r4u_tune.log 2>&1 || { tail -20 gpurun_out/r4u_tune.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4u_tune.log
