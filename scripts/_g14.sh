set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -u scripts/sched_ab.py --steps 300 --rounds 3 \
  --wide-variants "name=c2w_s40,15=3:40;name=c2w_s48,15=3:48;name=c2w_s56,15=3:56;name=c2w_s64,15=3:64;name=c2w_s48_c4w_mf6,15=3:48,11=14:6" > gpurun_out/ab15.log 2>&1
rc=$?; grep "us/step" gpurun_out/ab15.log; [ $rc -ne 0 ] && exit $rc
bash scripts/_g10.sh
