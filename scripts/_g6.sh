set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -u scripts/sched_ab.py --steps 300 --rounds 3 --cfg-variants "name=c2f_kw4,1=13:4;name=c2f_kw8,1=13:8;name=c3f_kw4,2=13:4;name=c3f_kw8,2=13:8;name=c3f_kw16,2=13:16;name=c4f_kw8,3=13:8;name=c4f_kw16,3=13:16;name=all_kw8,1=13:8,2=13:8,3=13:8" > gpurun_out/ab_kwave.log 2>&1
rc=$?; cat gpurun_out/ab_kwave.log | grep "us/step"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_kwave.log; exit $rc; }
bash scripts/_ab_so.sh "_C.so _C_epi2.so _C_epi3.so" 3 || exit 1
DDL_SO=_C_stamp.so timeout -k 10 200 python3 -u scripts/stamp_report.py --steps 4 > gpurun_out/stamps2.log 2>&1
rc=$?; head -12 gpurun_out/stamps2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/tta_calibrate.py "styles=1,noise=0.45,mix=0.25,shift=3,contrast=0.0" "styles=1,noise=0.55,mix=0.3,shift=3,contrast=0.2" "styles=2,noise=0.5,mix=0.3,shift=3,contrast=0.2" "styles=2,noise=0.6,mix=0.3,shift=4,contrast=0.3" "styles=1,noise=0.6,mix=0.35,shift=4,contrast=0.3" "styles=3,noise=0.5,mix=0.25,shift=3,contrast=0.2" "styles=2,noise=0.45,mix=0.25,shift=3,contrast=0.0" > gpurun_out/tta_cal2.log 2>&1
rc=$?; cat gpurun_out/tta_cal2.log; exit $rc
