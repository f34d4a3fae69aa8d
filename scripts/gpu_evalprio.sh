#!/bin/bash
# time-to-accuracy with training vs eval on the high-priority stream, alternating, one box
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/ab_combo.sh 3 "DDL_EVAL_PRIORITY=train" "DDL_EVAL_PRIORITY=eval" 2>&1 | tee gpurun_out/ab_evalprio.log
