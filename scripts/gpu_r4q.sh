#!/bin/bash
# Round 4: PMC default vs MF16 conv backward (item 1 evidence) + async step-end host latency.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
cd /tmp && export TMPDIR=/tmp
for mf in 0 1; do
  rm -rf $R/gpurun_out/pmc1_$mf $R/gpurun_out/pmc2_$mf
  DDL_PROBE_MF16=$mf timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc1_$mf -o pmc -- python3 $R/scripts/pmc_probe.py > $R/gpurun_out/pmc1_$mf.log 2>&1 || exit $?
  DDL_PROBE_MF16=$mf timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM TA_TA_BUSY GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc2_$mf -o pmc -- python3 $R/scripts/pmc_probe.py > $R/gpurun_out/pmc2_$mf.log 2>&1 || exit $?
  python3 $R/scripts/pmc_summary2.py $(find $R/gpurun_out/pmc1_$mf -name "*.db" | head -n 1) $(find $R/gpurun_out/pmc2_$mf -name "*.db" | head -n 1) > $R/gpurun_out/pmc_summary_$mf.txt 2>&1
  echo "== mf16=$mf"; cat $R/gpurun_out/pmc_summary_$mf.txt
done
rm -rf $R/gpurun_out/prof_async_rt
export DDL_TRACE=1
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace -d $R/gpurun_out/prof_async_rt -o prof -- python3 $R/bench.py --mode async --exchange xgmi --steps 60 --warmup 10 --tta 0 --prewarm-steps 20 > $R/gpurun_out/prof_async_rt.log 2>&1 || exit $?
unset DDL_TRACE
DB=$(find $R/gpurun_out/prof_async_rt -name "*.db" | head -n 1)
python3 $R/scripts/host_latency.py $DB --step 50 --tail 70 > $R/gpurun_out/latency_async.txt 2>&1
echo "== latency"; cat $R/gpurun_out/latency_async.txt | head -60
