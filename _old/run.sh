#!/usr/bin/env bash
# Reference: mnist_*/run.sh:3
#   mpiexec -n $1 python3 parameter_server.py -np $1 : -n $2 python3 worker.py -np $2
# MI355X: one process per GPU (W = num_workers), the P parameter-server shards
# co-located in them.  RCCL over xGMI carries gradient push / parameter pull.
#
# usage: bash run.sh <num_ps> <num_workers> [--variant mnist_sync_sharding_greedy] [flags...]
set -euo pipefail
NUM_PS=${1:?usage: run.sh <num_ps> <num_workers> [flags]}
NUM_WORKERS=${2:?usage: run.sh <num_ps> <num_workers> [flags]}
shift 2
cd "$(dirname "$0")"
export HSA_ENABLE_IPC_MODE_LEGACY=0
PORT=${MASTER_PORT:-$((29500 + RANDOM % 1000))}
exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$NUM_WORKERS" \
    --master-addr 127.0.0.1 --master-port "$PORT" \
    worker.py --num-ps "$NUM_PS" "$@"
