#!/bin/bash
# Every reference entry point / variant on one MI355X (W = 1), short epochs, reference print
# lines checked by eye in gpurun_out/entry_*.log.  Stops at the first failure.
set -u
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name, command...
  local n=$1; shift
  timeout -k 10 240 "$@" > gpurun_out/entry_$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(grep -c accuracy gpurun_out/entry_$n.log) accuracy lines; $(tail -2 gpurun_out/entry_$n.log | tr '\n' ' ' | cut -c1-150)"
  [ $rc -eq 0 ] || exit $rc
}
run single python single.py --steps 40
for v in mnist_sync mnist_async mnist_sync_sharding mnist_async_sharding mnist_sync_sharding_greedy mnist_async_sharding_greedy; do
  run $v python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 worker.py --variant $v --steps 40
done
run runsh bash run.sh 1 1 --steps 40 --eval-async
run ckpt python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 worker.py --steps 30 --checkpoint-dir gpurun_out/ck --checkpoint-every 10
run resume python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 worker.py --steps 30 --checkpoint-dir gpurun_out/ck --resume
run bench_async python bench.py --mode async --steps 50 --tta 0
run bench_contig python bench.py --shard contiguous --steps 50 --tta 0
run bench_greedy python bench.py --shard greedy --steps 50 --tta 0
