#!/bin/bash
# Async PS benches: W = 1 (RCCL-pair exchange vs xGMI exchange), W = 2 on one GPU (rehearsal).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for ex in rccl xgmi; do
  timeout -k 10 150 python bench.py --mode async --exchange $ex --steps 200 --warmup 20 --tta 0 \
      > gpurun_out/async_w1_$ex.log 2>&1
  rc=$?; echo "W=1 async $ex rc=$rc"; tail -1 gpurun_out/async_w1_$ex.log | cut -c1-330
  [ $rc -ne 0 ] && exit $rc
done
DDL_DIST_BACKEND=gloo timeout -k 10 150 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29433 bench.py --gpus 2 \
    --mode async --steps 50 --warmup 10 > gpurun_out/async_w2_shared.log 2>&1
rc=$?; echo "W=2 async shared rc=$rc"; tail -1 gpurun_out/async_w2_shared.log | cut -c1-330
exit $rc
