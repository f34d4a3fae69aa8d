set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
BENCH_ARGS="--force-collectives --exchange xgmi" bash scripts/gpu.sh timeline > /dev/null 2>&1 || exit 1
cp gpurun_out/timeline.txt gpurun_out/timeline_fx.txt; head -30 gpurun_out/timeline_fx.txt
BENCH_ARGS="--force-collectives --exchange rccl" bash scripts/gpu.sh timeline > /dev/null 2>&1 || exit 1
cp gpurun_out/timeline.txt gpurun_out/timeline_fr.txt; head -30 gpurun_out/timeline_fr.txt
