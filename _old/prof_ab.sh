#!/bin/bash
set -u
cd /root/repo
export TMPDIR=/tmp
R=$PWD
rm -rf gpurun_out/pold gpurun_out/pnew
(cd _old && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pold -o p -- python3 bench.py --steps 200 --warmup 20 --tta 0 --shard contiguous > /dev/null 2>&1) || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pnew -o p -- python3 bench.py --steps 200 --warmup 20 --tta 0 --shard contiguous > /dev/null 2>&1 || exit 1
find gpurun_out/pold gpurun_out/pnew -name "*kernel_stats.csv"
