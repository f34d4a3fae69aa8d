set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python3 -u scripts/sched_ab.py --steps 300 --rounds 2 --cfg-variants "1=0:2;1=0:4;1=0:8;1=2:2;1=2:4;1=2:8;1=4:2;1=4:4;1=4:8;1=6:2;1=6:4;1=6:8;1=7:2;1=7:4;1=7:8;2=0:2;2=0:4;2=0:8;2=2:2;2=2:4;2=2:8;2=4:2;2=4:4;2=4:8;2=6:2;2=6:4;2=6:8;2=7:2;2=7:4;2=7:8;3=0:2;3=0:4;3=0:8;3=2:2;3=2:4;3=2:8;3=4:2;3=4:4;3=4:8;3=6:2;3=6:4;3=6:8;3=7:2;3=7:4;3=7:8" > gpurun_out/ab13.log 2>&1
rc=$?; grep "us/step\|Error\|error" gpurun_out/ab13.log | head -60; exit $rc
