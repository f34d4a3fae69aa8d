#!/bin/bash
# two more passes of the real-step schedule tuner (longer timing windows)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u scripts/runner_tune.py --passes 2 --steps 800 --json gpurun_out/rtune2.json > gpurun_out/rtune2.log 2>&1
rc=$?; tail -40 gpurun_out/rtune2.log; exit $rc
