#!/bin/bash
# Multi-process rehearsal of the W > 1 benchmark on ONE GPU: W ranks share the card, the default
# process group runs over gloo, the data plane is the xGMI peer-memory exchange (RCCL refuses two
# ranks on one device).  Functional check of bench.py's W > 1 path (A/B, timing max over ranks,
# distributed eval, time-to-accuracy) - the numbers are not multi-GPU measurements.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp DDL_DIST_BACKEND=gloo DDL_XGMI_TIMEOUT_S=30
for W in ${WS:-2 4}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
      --master-addr 127.0.0.1 --master-port $((29400 + W)) bench.py --gpus $W \
      --steps ${STEPS:-50} --warmup 10 > gpurun_out/rehearsal_w$W.log 2>&1
  rc=$?; echo "W=$W rc=$rc"; tail -2 gpurun_out/rehearsal_w$W.log | cut -c1-600
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_n1.log 2>&1
rc=$?; echo "N=1 rc=$rc"; tail -1 gpurun_out/bench_n1.log | cut -c1-400
exit $rc
