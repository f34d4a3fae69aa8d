#!/bin/bash
# Round 4: bench.py at W = 4 as four processes on one GPU (sync xGMI exchange with READY
# flags; async xGMI data plane with push tails + gate), final tree.  Functional rehearsal of
# the driver's N = 4 run, not a multi-GPU measurement.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DDL_DIST_BACKEND=gloo
export DDL_DEBUG_DUMP_S=150
run() {  # label, port, bench args...
  local l=$1 p=$2; shift 2
  timeout -k 10 280 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
      --master-port $p scripts/bench_debug.py --gpus 4 "$@" > gpurun_out/r4ag_$l.log 2>&1
  local rc=$?; echo "$l rc=$rc"
  grep -v amdgpu.ids gpurun_out/r4ag_$l.log | tail -2 | cut -c1-900
  return $rc
}
run sync 29631 --steps 50 --warmup 10 --extra-plans "" && \
run async 29632 --mode async --steps 50 --warmup 10 --extra-plans ""
