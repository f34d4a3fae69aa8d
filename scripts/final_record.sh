# Final-record GPU run: the GPU suite, smoke(), the headline bench (300-step windows and the
# driver command), the async / forced-collective / contiguous variants, kernel stats, the step
# timeline and per-block stamps -> gpurun_out/final_record.log (+ logs).  usage (GPU box):
#   bash scripts/final_record.sh
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
L=gpurun_out/final_record.log
: > $L
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/t_all.log 2>&1
rc=$?; tail -1 gpurun_out/t_all.log | tee -a $L; [ $rc -ne 0 ] && { grep -B5 -A40 "FAIL\|Error" gpurun_out/t_all.log | head -80; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo "smoke ok: $(tail -1 gpurun_out/smoke.log)" | tee -a $L
one() {  # one <label> <seconds> <bench args...>
  local lab=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u bench.py "$@" > gpurun_out/fr.log 2>&1 || { echo "FAIL $lab"; tail -20 gpurun_out/fr.log; exit 1; }
  python3 - "$lab" "$*" >> $L <<'PY'
import json, sys
d = json.loads(open("gpurun_out/fr.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s} {d['ms_per_step']:.4f} ms/step  {d['value']:>10.1f} img/s  exchange={d['config'].get('exchange')}  args=[{sys.argv[2]}]")
PY
  tail -1 $L
}
for i in 1 2 3; do one "bench-300" 150 --steps 300 --warmup 20 --tta 0; done
for i in 1 2; do one "driver-cmd" 300 --gpus 1 --steps 20 --warmup 5; cp gpurun_out/fr.log gpurun_out/driver_cmd_$i.json; done
one "async-xgmi-w1-inline" 150 --steps 300 --warmup 20 --tta 0 --mode async --exchange xgmi
DDL_ASYNC_INLINE=0 one "async-xgmi-w1-service" 150 --steps 300 --warmup 20 --tta 0 --mode async --exchange xgmi
one "forced-xgmi" 200 --steps 300 --warmup 20 --tta 0 --force-collectives --exchange xgmi
one "forced-rccl" 200 --steps 300 --warmup 20 --tta 0 --force-collectives --exchange rccl
one "contiguous-plan" 150 --steps 300 --warmup 20 --tta 0 --shard contiguous
bash scripts/gpu.sh stats > gpurun_out/stats_run.log 2>&1 || { tail -20 gpurun_out/stats_run.log; exit 1; }
bash scripts/gpu.sh timeline > /dev/null 2>&1 || exit 1
head -16 gpurun_out/timeline.txt
DDL_SO=_C_stamp.so timeout -k 10 200 python3 -u scripts/stamp_report.py --steps 2 > gpurun_out/stamps_final.log 2>&1 || exit 1
head -14 gpurun_out/stamps_final.log
