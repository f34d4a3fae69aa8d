#!/bin/bash
# Round 4: bench.py at W = 2 as two processes on one GPU (gloo default group, xGMI data plane),
# with a stack dump if it stalls.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DDL_DIST_BACKEND=gloo
export DDL_DEBUG_DUMP_S=150
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29613 scripts/bench_debug.py --gpus 2 --steps 50 --warmup 10 --extra-plans "" > gpurun_out/r4w_bench_w2.log 2>&1
echo "rc=$?"
grep -v amdgpu.ids gpurun_out/r4w_bench_w2.log | tail -60
