set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/t_all.log 2>&1
rc=$?; tail -3 gpurun_out/t_all.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAIL\|Error" gpurun_out/t_all.log | head -80; exit $rc; }
for i in 1 2 3; do timeout -k 10 150 python3 -u bench.py --steps 300 --warmup 20 --tta 0 > gpurun_out/b11.log 2>&1 || exit 1; python3 -c "import json; print('300-step', json.loads(open('gpurun_out/b11.log').read().strip().splitlines()[-1])['ms_per_step'])"; done
for i in 1 2; do timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b11d.log 2>&1 || exit 1; python3 -c "import json; print('driver', json.loads(open('gpurun_out/b11d.log').read().strip().splitlines()[-1])['ms_per_step'])"; done
bash scripts/gpu.sh timeline > /dev/null 2>&1; rc=$?; head -16 gpurun_out/timeline.txt; [ $rc -ne 0 ] && exit $rc
DDL_SO=_C_stamp.so timeout -k 10 200 python3 -u scripts/stamp_report.py --steps 2 > gpurun_out/stamps4.log 2>&1
rc=$?; head -14 gpurun_out/stamps4.log; exit $rc
