set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
B=20480
timeout -k 10 600 python3 -u scripts/sched_ab.py --steps 300 --rounds 3 \
  --wide-variants "name=c4i6,10=3:6,10=inl;name=c4i6_c3s6,10=3:6,10=inl,12=3:6;name=c4i6_bf,10=3:6,10=inl,bf=$B;name=c4i6_c3s6_bf,10=3:6,10=inl,12=3:6,bf=$B;name=c4i8_c3s6_bf,10=3:8,10=inl,12=3:6,bf=$B;name=c4i6_c3s6_bf4,10=3:6,10=inl,12=3:6,bf=21504;name=c4i4_c3s6_bf,10=3:4,10=inl,12=3:6,bf=$B;name=c4i6_c3s6_c3w8_bf,10=3:6,10=inl,12=3:6,13=3:8,bf=$B;name=c4i6_c3s6_c3w16_bf,10=3:6,10=inl,12=3:6,13=3:16,bf=$B;name=c4i6_c3s5_bf,10=3:5,10=inl,12=3:5,bf=$B" > gpurun_out/ab9.log 2>&1
rc=$?; grep "us/step" gpurun_out/ab9.log; exit $rc
