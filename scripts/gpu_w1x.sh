#!/bin/bash
# W = 1 rehearsals of the W > 1 step: local update vs RCCL 1-rank vs xGMI push-to-self,
# alternating pairs on one box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -m pytest tests/test_native_runner.py -x -q -p no:cacheprovider -k forced > gpurun_out/w1x_tests.log 2>&1
rc=$?; tail -1 gpurun_out/w1x_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  for v in "local:" "rccl:--force-collectives --exchange rccl" "xgmi:--force-collectives --exchange xgmi"; do
    n=${v%%:*}; args=${v#*:}
    timeout -k 10 120 python bench.py --tta 0 --steps 300 $args > gpurun_out/w1x_$n.log 2>&1 || exit $?
    echo "$n $(tail -1 gpurun_out/w1x_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["exchange"])')"
  done
done
