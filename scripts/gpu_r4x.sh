#!/bin/bash
# Round 4: normal-priority training stream for the side-stream eval + gate guards: GPU suites
# touching the runners and the eval, W = 2 one-card bench with time-to-accuracy.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_native_runner.py tests/test_xgmi_gpu.py tests/test_gpu_trainer.py -x -v -m gpu -p no:cacheprovider \
    --timeout 240 --timeout-method thread > gpurun_out/r4x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r4x_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4x_tests.log | head; exit $rc; }
export DDL_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29617 bench.py --gpus 2 --steps 50 --warmup 10 --extra-plans "" > gpurun_out/r4x_bench_w2.log 2>&1 || { tail -30 gpurun_out/r4x_bench_w2.log; exit 1; }
tail -1 gpurun_out/r4x_bench_w2.log | cut -c1-300
