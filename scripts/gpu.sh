#!/bin/bash
# One parameterised GPU-box command for gpurun (replaces the per-experiment lease scripts of
# rounds 1-4, whose commands and outputs are recorded in docs/DESIGN.md and profiles/).
#
#   gpurun -- 'bash scripts/gpu.sh TIER [TIER ...]'
#
# Tiers run in order, each under its own time limit, and the script stops at the first failure
# (a GPU fault, abort or timeout ends the call: nothing else is started on the GPU after it).
#   tests      pytest -m gpu (the driver's round-end tier)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (the driver's 1-GPU command) -> gpurun_out/bench.json.log
#   tune       scripts/runner_tune.py --dma on the conv GEMMs  -> gpurun_out/tune.{log,json}
#   stats      rocprofv3 --kernel-trace --stats of a 200-step bench -> gpurun_out/stats_*.csv
#   timeline   rocprofv3 kernel trace + scripts/step_timeline.py -> gpurun_out/timeline.txt
#   pmc        two rocprofv3 --pmc passes (stall split, instruction mix, TA) over
#              scripts/pmc_probe.py + a TCC pass -> gpurun_out/pmc_summary.txt
#   sched      scripts/sched_ab.py with $SCHED_ARGS -> gpurun_out/sched.log
# Extra environment: BENCH_ARGS (bench / stats / timeline), TEST_ARGS (tests).
set -u
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {  # run <seconds> <log> <cmd...>
  local t=$1 log=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  tail -n 25 "$log"
  if [ $rc -ne 0 ]; then
    echo "[gpu.sh] '$*' failed rc=$rc (log $log)"
    exit $rc
  fi
}

for tier in "$@"; do
  echo "[gpu.sh] == $tier"
  case "$tier" in
    tests)
      run 900 gpurun_out/gpu_tests.log python3 -u -m pytest -m gpu -x -v --timeout 120 \
        --timeout-method thread ${TEST_ARGS:-} tests ;;
    smoke)
      run 300 gpurun_out/smoke.log python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run 600 gpurun_out/bench.json.log python3 -u bench.py ${BENCH_ARGS:-} ;;
    tune)
      run 1000 gpurun_out/tune.log python3 -u scripts/runner_tune.py --dma --passes 2 \
        --steps 200 --ops ${TUNE_OPS:-1,2,3,10,11,12,13,14,15} --json gpurun_out/tune.json ;;
    sched)
      run 600 gpurun_out/sched.log python3 -u scripts/sched_ab.py ${SCHED_ARGS:-} ;;
    stats)
      rm -rf gpurun_out/prof_stats
      (cd /tmp && TMPDIR=/tmp run 400 $R/gpurun_out/stats.log rocprofv3 --kernel-trace --stats \
        --output-format csv -d $R/gpurun_out/prof_stats -o prof -- \
        python3 $R/bench.py --steps 200 --warmup 10 --tta 0 ${BENCH_ARGS:-}) || exit $?
      for f in $(find gpurun_out/prof_stats -name "*stats*.csv"); do cp "$f" gpurun_out/; done
      find gpurun_out/prof_stats -name "*.db" -delete ;;
    timeline)
      rm -rf gpurun_out/prof_tl
      (cd /tmp && TMPDIR=/tmp run 400 $R/gpurun_out/timeline_run.log rocprofv3 --kernel-trace \
        -d $R/gpurun_out/prof_tl -o prof -- \
        python3 $R/bench.py --steps 60 --warmup 10 --tta 0 ${BENCH_ARGS:-}) || exit $?
      db=$(find gpurun_out/prof_tl -name "*.db" | head -n 1)
      python3 scripts/step_timeline.py "$db" > gpurun_out/timeline.txt 2>&1
      head -n 40 gpurun_out/timeline.txt
      find gpurun_out/prof_tl -name "*.db" -delete ;;
    pmc)
      rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
      (cd /tmp && TMPDIR=/tmp run 120 $R/gpurun_out/pmc1.log rocprofv3 --kernel-trace --pmc \
        SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
        SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE \
        -d $R/gpurun_out/pmc1 -o pmc -- python3 $R/scripts/pmc_probe.py) || exit $?
      (cd /tmp && TMPDIR=/tmp run 120 $R/gpurun_out/pmc2.log rocprofv3 --kernel-trace --pmc \
        SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT \
        SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM TA_TA_BUSY GRBM_GUI_ACTIVE \
        -d $R/gpurun_out/pmc2 -o pmc -- python3 $R/scripts/pmc_probe.py) || exit $?
      (cd /tmp && TMPDIR=/tmp run 120 $R/gpurun_out/pmc3.log rocprofv3 --kernel-trace --pmc \
        TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
        -d $R/gpurun_out/pmc3 -o pmc -- python3 $R/scripts/pmc_probe.py) || exit $?
      python3 scripts/pmc_summary2.py $(find gpurun_out/pmc1 -name "*.db" | head -n 1) \
        $(find gpurun_out/pmc2 -name "*.db" | head -n 1) > gpurun_out/pmc_summary.txt 2>&1
      python3 scripts/pmc_mem_summary.py $(find gpurun_out/pmc3 -name "*.db" | head -n 1) \
        > gpurun_out/pmc_l2.txt 2>&1
      cat gpurun_out/pmc_summary.txt gpurun_out/pmc_l2.txt | cut -c1-170
      find gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 -name "*.db" -delete ;;
    *)
      echo "[gpu.sh] unknown tier $tier"; exit 2 ;;
  esac
done
