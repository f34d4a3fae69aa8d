# usage: bash scripts/ab_so.sh "so1 so2 ..." ROUNDS [bench args]  (A/B of in-tree builds)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
SOS=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for so in $SOS; do
    DDL_SO=$so timeout -k 10 120 python3 -u bench.py --steps 300 --warmup 20 --tta 0 "$@" > gpurun_out/ab_$so.log 2>&1 || { echo "FAIL $so"; tail -5 gpurun_out/ab_$so.log; exit 1; }
    echo "$r $so $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$so.log').read().strip().splitlines()[-1]); print(d['ms_per_step'])")"
  done
done
