#!/bin/bash
# Round 4: gate guards with the null stream: forced / async benches, W = 2 one-card bench, and
# what the runtime reports for the streams' priorities.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -c "
import torch, ctypes
s = torch.cuda.current_stream()
print('current stream handle', s.cuda_stream, 'priority', s.priority, 'range', torch.cuda.Stream.priority_range())
for p in (-1, 0, 1):
    t = torch.cuda.Stream(priority=p); print('asked', p, 'got', t.priority)
" 2>&1 | grep -v amdgpu.ids
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r4y_b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/r4y_b_$l.log; exit 1; }
  tail -1 gpurun_out/r4y_b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], d['config']['parallelism'])"
}
b local --steps 300 --warmup 20 --tta 0
b forced_xgmi --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
b forced_rccl --steps 300 --warmup 20 --tta 0 --force-collectives
b async_xgmi --mode async --exchange xgmi --steps 300 --warmup 20 --tta 0
export DDL_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29619 bench.py --gpus 2 --steps 50 --warmup 10 --extra-plans "" > gpurun_out/r4y_bench_w2.log 2>&1 || { tail -30 gpurun_out/r4y_bench_w2.log; exit 1; }
tail -1 gpurun_out/r4y_bench_w2.log | cut -c1-200
