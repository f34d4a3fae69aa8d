"""Model: tensor layout, torch oracle engine, HIP engine."""
from __future__ import annotations

import torch

from .layout import TENSORS, NUM_TENSORS, TOTAL_NUMEL  # noqa: F401

# Backward segments of the HIP engine in completion order (fc head first), each the set
# of tensors whose gradients are final when the segment's kernels have run
# (SURVEY.md §5.8 bucket plan, refined per conv layer).  fc1 / fc2's weight gradients run in
# the conv4 dual launch (csrc/kernels/engine_impl.h FcWgradAux), so they complete with segment 1.
HIP_SEGMENTS = [[12, 13], [6, 7, 8, 9, 10, 11], [4, 5], [0, 1, 2, 3]]
TORCH_SEGMENTS = [list(range(14))]


def resolve_engine(kind: str, device) -> str:
    device = torch.device(device)
    if kind == "auto":
        return "hip" if device.type == "cuda" else "torch"
    if kind == "hip" and device.type != "cuda":
        raise ValueError("the HIP engine needs a GPU device")
    return kind


def engine_segments(kind: str, device):
    return HIP_SEGMENTS if resolve_engine(kind, device) == "hip" else TORCH_SEGMENTS


def make_engine(kind: str, params, grads, offsets, device, batch: int = 100, graph: bool = True):
    kind = resolve_engine(kind, device)
    if kind == "hip":
        from .hip_engine import HipEngine
        return HipEngine(params, grads, offsets, batch=batch, graph=graph)
    from .mnist_cnn import TorchEngine
    return TorchEngine(params, grads, offsets, batch=batch)
