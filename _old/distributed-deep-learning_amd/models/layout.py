"""Static tensor table of the MNIST CNN.

Reference: the 14 trainable variables ``mnist/v0`` .. ``mnist/v13`` created in
``mnist_sync/model/model.py:24-86`` and listed (in that order) by
``trainable_variables()`` at ``mnist_sync/model/model.py:96-98``.  The reference ships
this table from one worker to every PS as a pickled metadata dict
(``mnist_sync_sharding/worker.py:71-75``); here every rank computes it statically, so
no metadata exchange is needed.

Canonical flat order is v0..v13.  Every layer's weight is immediately followed by its
bias, so each layer is an *augmented* matrix ``[K_in + 1, C_out]`` in the flat buffer
(weights HWIO-flattened to ``[K_in, C_out]``, bias as the extra row).  The HIP kernels
exploit this: a weight-gradient GEMM with a row of ones appended to its left operand
writes dW and db in one pass.
"""
from __future__ import annotations

from dataclasses import dataclass
from math import prod
from typing import List, Tuple

IMAGE = 28
NUM_CLASSES = 10
INPUT_DIM = IMAGE * IMAGE


@dataclass(frozen=True)
class TensorSpec:
    index: int
    name: str           # "v0" .. "v13" (reference variable names)
    shape: Tuple[int, ...]
    layer: str          # conv1..conv4, fc1..fc3
    kind: str           # "weight" | "bias"

    @property
    def numel(self) -> int:
        return prod(self.shape)

    @property
    def nbytes(self) -> int:
        return 4 * self.numel


_SHAPES = [
    ((5, 5, 1, 32), "conv1", "weight"),     # model.py:24
    ((32,), "conv1", "bias"),               # model.py:26
    ((5, 5, 32, 64), "conv2", "weight"),    # model.py:35
    ((64,), "conv2", "bias"),               # model.py:37
    ((5, 5, 64, 128), "conv3", "weight"),   # model.py:46
    ((128,), "conv3", "bias"),              # model.py:48
    ((5, 5, 128, 256), "conv4", "weight"),  # model.py:57
    ((256,), "conv4", "bias"),              # model.py:59
    ((1024, 1024), "fc1", "weight"),        # model.py:67
    ((1024,), "fc1", "bias"),               # model.py:68
    ((1024, 512), "fc2", "weight"),         # model.py:77
    ((512,), "fc2", "bias"),                # model.py:78
    ((512, 10), "fc3", "weight"),           # model.py:85
    ((10,), "fc3", "bias"),                 # model.py:86
]

TENSORS: List[TensorSpec] = [
    TensorSpec(i, f"v{i}", s, layer, kind) for i, (s, layer, kind) in enumerate(_SHAPES)
]
NUM_TENSORS = len(TENSORS)
TOTAL_NUMEL = sum(t.numel for t in TENSORS)          # 2,656,010
TOTAL_BYTES = 4 * TOTAL_NUMEL                        # 10,624,040

# Canonical (v0..v13) element offsets.
CANON_OFFSETS: List[int] = []
_o = 0
for _t in TENSORS:
    CANON_OFFSETS.append(_o)
    _o += _t.numel
del _o, _t

# Conv geometry per layer: (H_in, C_in, C_out, H_pool) with SAME 5x5 conv and
# SAME 2x2/2 max-pool (model.py:28-31, 39-42, 50-53, 61-64).
CONV_LAYERS = [
    # name,   H,  Cin, Cout, Hp
    ("conv1", 28, 1, 32, 14),
    ("conv2", 14, 32, 64, 7),
    ("conv3", 7, 64, 128, 4),
    ("conv4", 4, 128, 256, 2),
]
FC_LAYERS = [
    ("fc1", 1024, 1024),
    ("fc2", 1024, 512),
    ("fc3", 512, 10),
]


def tensor_names(scope: str = "mnist") -> List[str]:
    """Fully-qualified variable names as TF would print them."""
    return [f"{scope}/{t.name}" for t in TENSORS]


def forward_flops_per_sample() -> int:
    """Forward FLOPs/sample (2 x MACs), SURVEY.md §2.6 = 70.77 MFLOP."""
    f = 0
    for _, h, cin, cout, _ in CONV_LAYERS:
        f += 2 * h * h * cout * 25 * cin
    for _, k, n in FC_LAYERS:
        f += 2 * k * n
    return f
