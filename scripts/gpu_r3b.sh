#!/bin/bash
# round 3: GPU suite without the 8-process cases, then those alone (each step time-limited;
# stops at the first failure), then the forced-rehearsal and async W=1 benches
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 240 \
    --timeout-method thread -k "not w8" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
if [ "${W8:-1}" = "1" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -x -v -m gpu -p no:cacheprovider \
      --timeout 300 --timeout-method thread -k "w8" > gpurun_out/gpu_tests_w8.log 2>&1
  rc=$?; echo "w8 tests rc=$rc"; tail -4 gpurun_out/gpu_tests_w8.log
  [ $rc -ne 0 ] && exit $rc
fi
out=gpurun_out/bench_r3b.log; : > $out
for cfg in "--force-collectives --exchange xgmi" "--force-collectives --exchange rccl" "--mode async" ""; do
  echo "== $cfg" >> $out
  timeout -k 10 120 python bench.py --steps 200 --tta 0 $cfg >> $out 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc ($cfg)"; tail -5 $out; exit $rc; }
done
python - <<'PY'
import json
cfg = None
for line in open("gpurun_out/bench_r3b.log"):
    if line.startswith("=="): cfg = line.strip()
    elif line.startswith("{"): r = json.loads(line); print(cfg, r["ms_per_step"], r["config"]["exchange"])
PY
