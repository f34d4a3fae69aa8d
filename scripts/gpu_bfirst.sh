#!/bin/bash
# dual launches: which problem's blocks dispatch first (DDL_DUAL_BFIRST bit per data-gradient op)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
bash scripts/ab_combo.sh 3 "DDL_DUAL_BFIRST=16384" "DDL_DUAL_BFIRST=20480" "DDL_DUAL_BFIRST=17408" "DDL_DUAL_BFIRST=0" 2>&1 | tee gpurun_out/ab_bfirst.log
