#!/bin/bash
# Round 4: are the released trainers really gone?  One-card W = 4 bench with DDL_BENCH_DEBUG.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DDL_DIST_BACKEND=gloo DDL_DEBUG_DUMP_S=120 DDL_BENCH_DEBUG=1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29681 scripts/bench_debug.py --gpus 4 --extra-plans "" --steps 20 --warmup 5 > gpurun_out/r4am.log 2>&1
rc=$?; echo "rc=$rc"; grep "trainer(s) alive" gpurun_out/r4am.log
grep '^{"metric"' gpurun_out/r4am.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print(d['time_to_acc']['epoch_wall_s'], d['time_to_acc_replicate']['epoch_wall_s'])"
exit $rc
