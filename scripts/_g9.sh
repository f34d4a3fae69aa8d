set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_xgmi_gpu.py -k "checkpoint or inline or serves_every_push and 1-" > gpurun_out/t_async.log 2>&1
rc=$?; tail -3 gpurun_out/t_async.log; [ $rc -ne 0 ] && { grep -B5 -A40 "FAIL\|Error" gpurun_out/t_async.log | head -80; exit $rc; }
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['config'].get('exchange'))" "$@"; }
for i in 1 2; do
  timeout -k 10 150 python3 -u bench.py --steps 300 --warmup 20 --tta 0 > gpurun_out/bs.log 2>&1 || exit 1; ms gpurun_out/bs.log sync
  timeout -k 10 150 python3 -u bench.py --steps 300 --warmup 20 --tta 0 --mode async --exchange xgmi > gpurun_out/ba.log 2>&1 || exit 1; ms gpurun_out/ba.log async-inline
  DDL_ASYNC_INLINE=0 timeout -k 10 150 python3 -u bench.py --steps 300 --warmup 20 --tta 0 --mode async --exchange xgmi > gpurun_out/ba0.log 2>&1 || exit 1; ms gpurun_out/ba0.log async-service
done
BENCH_ARGS="--mode async --exchange xgmi" bash scripts/gpu.sh timeline > /dev/null 2>&1; rc=$?; cp gpurun_out/timeline.txt gpurun_out/timeline_async.txt; head -18 gpurun_out/timeline.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python3 -u scripts/sched_ab.py --steps 300 --rounds 3 \
  --wide-variants "name=c4s5_c3s5_bf,10=3:5,10=inl,12=3:5,bf=20480;name=c4s6_c3s5_bf,10=3:6,10=inl,12=3:5,bf=20480;name=c4s4_c3s5_bf,10=3:4,10=inl,12=3:5,bf=20480;name=c4s5_c3s4_bf,10=3:5,10=inl,12=3:4,bf=20480;name=c4s5_c3s6_bf,10=3:6,10=inl,12=3:6,bf=20480;name=c4s5_c3s5_c2s3_bf,10=3:5,10=inl,12=3:5,14=14:3,bf=20480;name=c4s5_c3s5_c2s6_bf,10=3:5,10=inl,12=3:5,14=14:6,bf=20480;name=c4s5_c3s5_bf3,10=3:5,10=inl,12=3:5,bf=4096;name=c4s5_c3s5_c3w10_bf,10=3:5,10=inl,12=3:5,13=14:10,bf=20480;name=c4s5_c3s5_c4w6_bf,10=3:5,10=inl,12=3:5,11=14:6,bf=20480" > gpurun_out/ab10.log 2>&1
rc=$?; grep "us/step" gpurun_out/ab10.log; exit $rc
