#!/bin/bash
# Two PMC passes over default training steps (rocprofv3 --pmc with --kernel-trace only).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc1 $R/gpurun_out/pmc2
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc1 -o pmc -- python3 $R/scripts/pmc_probe.py > $R/gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM TA_TA_BUSY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc2 -o pmc -- python3 $R/scripts/pmc_probe.py > $R/gpurun_out/pmc2.log 2>&1 || exit $?
cd $R
python3 scripts/pmc_summary2.py $(find gpurun_out/pmc1 -name "*.db" | head -n 1) $(find gpurun_out/pmc2 -name "*.db" | head -n 1) > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt
