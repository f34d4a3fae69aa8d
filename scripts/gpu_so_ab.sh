#!/bin/bash
# Same-box A/B of two in-tree builds of the extension (DDL_SO), alternating runs, after the
# kernel numerics tests of the default build; then one kernel-trace timeline of the default.
#   SO_B=_C_ab.so bash scripts/gpu_so_ab.sh [rounds]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
ROUNDS=${1:-3}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_hip_kernels.py tests/test_native_runner.py} \
      -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
for i in $(seq $ROUNDS); do
  for so in _C.so ${SO_B:-_C_ab.so}; do  # SO_B may list several builds
    DDL_SO=$so timeout -k 10 120 python bench.py --tta 0 --steps 400 --warmup 40 ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || exit $?
    echo "$so $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
rm -rf gpurun_out/proft
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/proft -o prof -- python3 bench.py --steps 60 --warmup 10 --tta 0 ${BENCH_ARGS:-} > gpurun_out/proft.log 2>&1 || exit $?
python3 scripts/step_timeline.py $(find gpurun_out/proft -name "*.db" | head -n 1) --step 40 > gpurun_out/timeline_t.txt 2>&1 || exit $?
cat gpurun_out/timeline_t.txt
