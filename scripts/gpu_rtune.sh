#!/bin/bash
# real-step schedule tune (scripts/runner_tune.py), then bench with the engine defaults
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u scripts/runner_tune.py --passes ${PASSES:-2} --steps ${STEPS:-400} --json gpurun_out/rtune.json > gpurun_out/rtune.log 2>&1
rc=$?; tail -25 gpurun_out/rtune.log; exit $rc
