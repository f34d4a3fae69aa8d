"""Counter-based dropout RNG shared bit-for-bit by the HIP kernels and the torch oracle.

TF1 ``tf.nn.dropout(x, rate)`` (``mnist_sync/model/model.py:73-74,82``) keeps an element
when ``uniform[0,1) >= rate`` and scales kept elements by ``1/(1-rate)`` [TF-semantics].
We draw the uniform from a stateless hash of (seed, layer, element index) so that the
forward kernel, the backward kernel (which regenerates the mask instead of storing it)
and the CPU oracle all agree exactly.  The same constants appear in
``csrc/kernels/common.h`` (``ddl_hash32`` / ``ddl_keep``).
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF
GOLDEN = 0x9E3779B9


def _mix(x: torch.Tensor) -> torch.Tensor:
    # lowbias32 finalizer; x is int64 holding a uint32.
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & M32
    x = x ^ (x >> 16)
    return x


def mix_scalar(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def layer_key(seed: int, layer: int) -> int:
    return mix_scalar((seed + layer * GOLDEN) & M32)


def rate_threshold(keep_prob: float) -> int:
    """24-bit integer threshold: keep iff (hash >> 8) >= threshold."""
    rate = 1.0 - float(keep_prob)
    return int(round(rate * (1 << 24)))


def keep_mask(seed: int, layer: int, numel: int, keep_prob: float,
              device: torch.device | str = "cpu") -> torch.Tensor:
    """Boolean keep mask for ``numel`` elements (row-major element index)."""
    thr = rate_threshold(keep_prob)
    if thr <= 0:
        return torch.ones(numel, dtype=torch.bool, device=device)
    key = layer_key(seed, layer)
    idx = torch.arange(numel, dtype=torch.int64, device=device)
    h = _mix(idx ^ key)
    return (h >> 8) >= thr


def step_seed(base_seed: int, rank: int, step: int) -> int:
    """Per-(worker, step) dropout seed; workers draw different masks like the
    reference's independent TF RNGs."""
    return mix_scalar((base_seed * 1000003 + rank * 7919 + step * GOLDEN) & M32)
