#!/bin/bash
# Round 4: bench.py releases the earlier trainers before each W > 1 sync time-to-accuracy run.
# One-card W = 4 (default side-stream eval, then in line) and W = 2, plus the GPU bench tests.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -x -v -m gpu -k side_stream_eval \
    -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r4ak_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4ak_tests.log; [ $rc -ne 0 ] && exit $rc
export DDL_DIST_BACKEND=gloo
export DDL_DEBUG_DUMP_S=120
run() {  # label, nproc, port, bench args...
  local l=$1 n=$2 p=$3; shift 3
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $p scripts/bench_debug.py --gpus $n --extra-plans "" "$@" > gpurun_out/r4ak_$l.log 2>&1
  local rc=$?; echo "$l rc=$rc"
  [ $rc -eq 0 ] && grep '^{"metric"' gpurun_out/r4ak_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print(d['ms_per_step'], d['config']['parallelism'], d['config']['exchange'], d['time_to_acc'], d['time_to_acc_replicate'])"
  return $rc
}
run w4 4 29671 --steps 50 --warmup 10 && run w4_inline 4 29672 --steps 20 --warmup 5 --tta-sync-eval && \
run w2 2 29673 --steps 50 --warmup 10
