#!/bin/bash
# Round 4: MFMA 16x16x4 vs 32x32x2 peak, then kernel timelines of the default step and the
# conv backward on CFG_MF16 (rocprofv3 kernel trace, one step each).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
timeout -k 10 120 python scripts/mfma_peak.py > gpurun_out/r4b_peak.log 2>&1 || { cat gpurun_out/r4b_peak.log; exit 1; }
cat gpurun_out/r4b_peak.log
cd /tmp && export TMPDIR=/tmp
for v in default "bwd14 x2"; do
  tag=$(echo "$v" | tr -d ' ')
  rm -rf $R/gpurun_out/prof_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_$tag -o prof -- python3 $R/scripts/mf16_ab.py --profile "$v" --steps 80 > $R/gpurun_out/prof_$tag.log 2>&1 || exit $?
  python3 $R/scripts/step_timeline.py $(find $R/gpurun_out/prof_$tag -name "*.db" | head -n 1) --step 100 > $R/gpurun_out/timeline_$tag.txt 2>&1 || exit $?
  echo "== $v"; cat $R/gpurun_out/timeline_$tag.txt
done
