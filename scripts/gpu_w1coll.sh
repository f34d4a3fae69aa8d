#!/bin/bash
# Multi-GPU step structure rehearsed on one GPU: native-runner tests, then the bench with the
# exchange forced onto a 1-rank RCCL communicator, A/B of DDL_LAST_ON_MAIN (alternating runs),
# then the default bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_native_runner.py} -x -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/w1c_tests.log 2>&1 || { tail -20 gpurun_out/w1c_tests.log; exit 1; }
tail -2 gpurun_out/w1c_tests.log
for i in 1 2; do
  for v in ${VALS:-1 0}; do
    env ${VAR:-DDL_LAST_ON_MAIN}=$v timeout -k 10 120 python bench.py --steps 400 --warmup 40 --tta 0 \
      --force-collectives ${EXTRA:-} > gpurun_out/w1c_$v.log 2>&1 || { tail -5 gpurun_out/w1c_$v.log; exit 1; }
    python -c "import sys,json; d=json.loads(open('gpurun_out/w1c_$v.log').readlines()[-1]); print('forced ${VAR:-DDL_LAST_ON_MAIN}=$v', d['ms_per_step'], d['config']['exchange'])"
  done
done
timeout -k 10 120 python bench.py --steps 400 --warmup 40 --tta 0 > gpurun_out/w1c_default.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/w1c_default.log').readlines()[-1]); print('default W=1', d['ms_per_step'])"
