#!/bin/bash
# Round 4: bench.py --mode async at W = 2 as two processes on one GPU (xGMI async data plane,
# gate + board), with both time-to-accuracy runs (side-stream eval).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DDL_DIST_BACKEND=gloo
export DDL_DEBUG_DUMP_S=150
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29621 scripts/bench_debug.py --gpus 2 --mode async --steps 50 --warmup 10 --extra-plans "" > gpurun_out/r4ae_bench_w2_async.log 2>&1
rc=$?; echo "rc=$rc"
grep -v amdgpu.ids gpurun_out/r4ae_bench_w2_async.log | tail -3 | cut -c1-1200
exit $rc
