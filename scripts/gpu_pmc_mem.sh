#!/bin/bash
# One PMC pass of memory-hierarchy counters over default training steps (--kernel-trace only).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc3
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCR_TCP_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCC_HIT TCC_MISS TA_TA_BUSY TD_TD_BUSY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc3 -o pmc -- python3 $R/scripts/pmc_probe.py > $R/gpurun_out/pmc3.log 2>&1 || exit $?
cd $R
python3 scripts/pmc_mem_summary.py $(find gpurun_out/pmc3 -name "*.db" | head -n 1) > gpurun_out/pmc_mem_summary.txt 2>&1
cat gpurun_out/pmc_mem_summary.txt
