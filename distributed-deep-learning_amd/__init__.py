"""ddl_amd — MI355X-native parameter-server training framework.

Capabilities mirror epikjjh/DIstributed-Deep-Learning (six ``mnist_*`` variants:
sync/async parameter servers, single/contiguous/greedy sharding), re-designed for
MI355X: hand-written gfx950 HIP kernels for the CNN forward/backward and the fused
TF1-Adam shard update, a C++ step runner that enqueues the whole training step on one
stream (eager launches: replaying the step as a HIP graph measured slower, so graphs are
opt-in), RCCL (``torch.distributed`` backend ``nccl``) or our own xGMI peer-memory kernels
for gradient push / parameter pull, and a native shared-memory mailbox for the
asynchronous control plane.

Sub-packages:
  models/    layout table of the 14 tensors, the CNN (torch oracle + HIP engine)
  ops/       native extension loader, kernel wrappers, TF1 Adam, dropout hash
  parallel/  shard planners, communication plans, PS / worker roles, launcher
  utils/     data (mnist.pkl / npz / synthetic), metrics, checkpoint, tracing
"""
__version__ = "0.1.0"

import os as _os

# Kernel arguments in device memory (read by the dispatcher from HBM instead of host memory
# over the bus).  The step is ~17 dependent launches: host-resident kernargs measured
# 0.3255 vs 0.3045 ms/step (docs/DESIGN.md).  This ROCm defaults to device kernargs already;
# the setting pins it for any runtime whose default differs.  Must precede HIP init.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
# Cross-process GPU memory sharing (RCCL's P2P transports, the xGMI exchanges' IPC handles)
# through dmabuf: the MI355X hosts this runs on only support dmabuf IPC, and with the legacy
# mode hipIpcGetMemHandle fails ("invalid argument").  Every launcher script exports it; the
# setdefault covers a torchrun started without them (e.g. the driver's multi-GPU bench).
# Must precede HIP init.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

# Presets named after the reference's six variant directories
# (reference: mnist_*/run.sh:3).
VARIANTS = {
    "mnist_sync": dict(mode="sync", shard="none"),
    "mnist_async": dict(mode="async", shard="none"),
    "mnist_sync_sharding": dict(mode="sync", shard="contiguous"),
    "mnist_async_sharding": dict(mode="async", shard="contiguous"),
    "mnist_sync_sharding_greedy": dict(mode="sync", shard="greedy"),
    "mnist_async_sharding_greedy": dict(mode="async", shard="greedy"),
}
