# Time to accuracy (easy + hard synthetic sets) for sync / async at W = 1, and W = 2 / 4 as
# processes sharing one card (gloo rehearsal) -> gpurun_out/tta_w*.json.  usage: bash scripts/tta_runs.sh
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
summ() { python3 - "$@" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
def f(k):
    t = d.get(k)
    return "-" if not t else f"t95={t['time_to_target_s']} at-step={t.get('steps_to_target')} final={t['final_acc']}"
print(sys.argv[2], d["ms_per_step"], d["config"].get("exchange"), "| easy", f("time_to_acc"), "| easy-rep", f("time_to_acc_replicate"), "| hard", f("time_to_acc_hard"), "| hard-rep", f("time_to_acc_hard_replicate"))
PY
}
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > gpurun_out/tta_w1_sync.json 2>gpurun_out/tta_w1_sync.err || exit 1; summ gpurun_out/tta_w1_sync.json w1-sync
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --mode async --exchange xgmi > gpurun_out/tta_w1_async.json 2>gpurun_out/tta_w1_async.err || exit 1; summ gpurun_out/tta_w1_async.json w1-async-xgmi
port=29611
for W in 2 4; do for M in sync async; do
  port=$((port+7))
  DDL_DIST_BACKEND=gloo timeout -k 10 500 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $port bench.py --gpus $W --steps 50 --warmup 10 --mode $M > gpurun_out/tta_w${W}_$M.json 2>gpurun_out/tta_w${W}_$M.err || { tail -20 gpurun_out/tta_w${W}_$M.err; exit 1; }
  summ gpurun_out/tta_w${W}_$M.json w$W-$M
done; done
