set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_gpu_trainer.py > gpurun_out/t_kern.log 2>&1
rc=$?; tail -2 gpurun_out/t_kern.log; [ $rc -ne 0 ] && { grep -B5 -A30 "FAIL\|Error" gpurun_out/t_kern.log | head -60; exit $rc; }
bash scripts/_ab_so.sh "_C.so _C_headold.so" 3 || exit 1
timeout -k 10 700 python3 -u scripts/sched_ab.py --steps 300 --rounds 3 \
  --wide-variants "name=fc1_s4,4=3:4,4=inl;name=fc1_s8,4=3:8,4=inl;name=fc1_s16,4=3:16,4=inl;name=fc1_s32w,4=3:32,4=wide;name=c2f_s2,1=3:2;name=c2f_s4,1=3:4;name=c3f_s2,2=3:2;name=c3f_s4,2=3:4;name=c4f_s4,3=3:4;name=c4f_s8,3=3:8;name=fc2_s8,5=3:8;name=fc2_s32,5=3:32" > gpurun_out/ab12.log 2>&1
rc=$?; grep "us/step" gpurun_out/ab12.log; exit $rc
