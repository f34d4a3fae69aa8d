#!/bin/bash
# Round 4: W = 4 sync on one GPU, time-to-accuracy with the eval on the training stream
# (--tta-sync-eval) vs the side stream: is the slow one-card W = 4 TTA epoch a hardware-queue
# oversubscription artifact of four processes sharing one card?
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DDL_DIST_BACKEND=gloo
export DDL_DEBUG_DUMP_S=150
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29641 scripts/bench_debug.py --gpus 4 --steps 20 --warmup 5 --extra-plans "" --tta-sync-eval \
    > gpurun_out/r4ah_sync_evalsync.log 2>&1
rc=$?; echo "rc=$rc"
grep '^{"metric"' gpurun_out/r4ah_sync_evalsync.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print(d['ms_per_step'], d['time_to_acc'], d.get('time_to_acc_replicate'))"
exit $rc
