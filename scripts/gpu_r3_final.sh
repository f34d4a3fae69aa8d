#!/bin/bash
# Round-3 record on one box: GPU suite, smoke, the driver's bench command, longer windows,
# forced W > 1 rehearsals (RCCL / xGMI), async W = 1, every entry point.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
out=gpurun_out/final_record.log
: > $out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/gpu_tests_final.log)" | tee -a $out
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/smoke.log)" | tee -a $out
[ $rc -ne 0 ] && exit $rc
b() {  # label, bench args...
  local l=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/b_$l.log 2>&1 || { echo "bench $l failed"; tail -5 gpurun_out/b_$l.log; exit 1; }
  tail -1 gpurun_out/b_$l.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); t = d.get('time_to_acc') or {}
print('$l', d['value'], d['ms_per_step'], d['config']['exchange'], 'tta', t.get('time_to_target_s'), 'final', t.get('final_acc'))" | tee -a $out
}
for r in 1 2; do
  b driver$r --gpus 1 --steps 20 --warmup 5
  b w300_$r --steps 300 --warmup 20 --tta 0
done
b forced_rccl --steps 300 --warmup 20 --tta 0 --force-collectives
b forced_xgmi --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
b async_w1 --mode async --steps 300 --warmup 20 --tta 0
b contig --shard contiguous --steps 300 --warmup 20 --tta 0
bash scripts/gpu_entrypoints.sh 2>&1 | tee -a $out
