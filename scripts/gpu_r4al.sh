#!/bin/bash
# Round 4: rocprofv3 kernel stats of the default 1-GPU bench step on the final tree.
set -u
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o prof -- python3 $R/bench.py --steps 200 --warmup 10 --tta 0 > $R/gpurun_out/prof_stats.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $R/gpurun_out/prof_stats.log | cut -c1-300
find $R/gpurun_out/prof_stats -name "*.csv" | sed "s|$R/||"
for f in $(find $R/gpurun_out/prof_stats -name "*stats*.csv"); do cp $f $R/gpurun_out/r4al_$(basename $f); done
find $R/gpurun_out/prof_stats -name "*.db" -delete
exit $rc
