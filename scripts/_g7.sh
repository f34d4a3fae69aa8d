set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_native_runner.py > gpurun_out/t_kern.log 2>&1
rc=$?; tail -3 gpurun_out/t_kern.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAIL\|Error" gpurun_out/t_kern.log | head -60; exit $rc; }
for i in 1 2 3; do timeout -k 10 120 python3 -u bench.py --steps 300 --warmup 20 --tta 0 > gpurun_out/b7.log 2>&1 || exit 1; python3 -c "import json; print(json.loads(open('gpurun_out/b7.log').read().strip().splitlines()[-1])['ms_per_step'])"; done
bash scripts/gpu.sh timeline > /dev/null 2>&1; rc=$?; head -16 gpurun_out/timeline.txt; [ $rc -ne 0 ] && exit $rc
DDL_SO=_C_stamp.so timeout -k 10 200 python3 -u scripts/stamp_report.py --steps 2 > gpurun_out/stamps3.log 2>&1
rc=$?; head -12 gpurun_out/stamps3.log; exit $rc
