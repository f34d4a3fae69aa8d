"""TF1 Adam on a flat parameter shard (plus SGD / momentum).

Reference: ``tf.compat.v1.train.AdamOptimizer(1e-4)`` created on every PS
(``mnist_sync/parameter_server.py:21,26-27``; sharded
``mnist_sync_sharding/parameter_server.py:63-69``) and in the single trainer via
``minimize`` (``mnist_sync/model/model.py:93,106``).  TF1 semantics [TF-semantics]::

    t      += 1                                   (beta1_power = beta1**t)
    lr_t    = lr * sqrt(1 - beta2**t) / (1 - beta1**t)
    m       = beta1*m + (1-beta1)*g
    v       = beta2*v + (1-beta2)*g*g
    w      -= lr_t * m / (sqrt(v) + eps)           ("epsilon hat" form)

Each PS keeps its *own* step counter (``beta1_power``/``beta2_power`` per PS graph),
which matters in async mode where PSes advance at different rates.

On GPU the update is one fused HIP kernel over the owned shard (``adam_flat`` in
``csrc/kernels/optim.hip``); the torch path below is the CPU implementation and the
test oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from . import native


@dataclass
class AdamHyper:
    lr: float = 1e-4
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8


def adam_coeffs(h: AdamHyper, t: int):
    """Host-side scalars for step t (1-based)."""
    lr_t = h.lr * math.sqrt(1.0 - h.beta2 ** t) / (1.0 - h.beta1 ** t)
    return lr_t


def adam_torch_(w: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                h: AdamHyper, t: int, grad_scale: float = 1.0) -> None:
    lr_t = adam_coeffs(h, t)
    if grad_scale != 1.0:
        g = g * grad_scale
    # TF ApplyAdam form: m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2)
    m.add_((g - m) * (1.0 - h.beta1))
    v.add_((g * g - v) * (1.0 - h.beta2))
    w.sub_(lr_t * m / (v.sqrt() + h.eps))


class FlatAdam:
    """Adam state for one contiguous shard ``[lo, hi)`` of a flat parameter buffer.

    ``step(params, grads)`` takes the *full* flat buffers (or shard views) and updates
    ``params[lo:hi]`` in place from ``grads[lo:hi]``.
    """

    def __init__(self, numel: int, device, hyper: AdamHyper | None = None,
                 optimizer: str = "adam", momentum: float = 0.9):
        self.h = hyper or AdamHyper()
        self.numel = numel
        self.t = 0
        self.optimizer = optimizer
        self.momentum = momentum
        self.m = torch.zeros(numel, dtype=torch.float32, device=device)
        self.v = (torch.zeros(numel, dtype=torch.float32, device=device)
                  if optimizer == "adam" else None)

    def step(self, w: torch.Tensor, g: torch.Tensor, grad_scale: float = 1.0) -> None:
        assert w.numel() == self.numel and g.numel() == self.numel
        self.t += 1
        use_native = w.is_cuda and native.available()
        if self.optimizer == "adam":
            if use_native:
                native.ops().adam_flat(w, g, self.m, self.v, adam_coeffs(self.h, self.t),
                                       self.h.beta1, self.h.beta2, self.h.eps, grad_scale)
            else:
                adam_torch_(w, g, self.m, self.v, self.h, self.t, grad_scale)
        elif self.optimizer == "momentum":
            if use_native:
                native.ops().momentum_flat(w, g, self.m, self.h.lr, self.momentum, grad_scale)
            else:
                self.m.mul_(self.momentum).add_(g, alpha=grad_scale)
                w.sub_(self.h.lr * self.m)
        elif self.optimizer == "sgd":
            w.sub_(g, alpha=self.h.lr * grad_scale)
        else:
            raise ValueError(self.optimizer)

    # ---- checkpoint helpers (TF1 slot naming) -------------------------
    def state_tensors(self):
        out = {"Adam": self.m}
        if self.v is not None:
            out["Adam_1"] = self.v
        return out

    def powers(self):
        return self.h.beta1 ** self.t, self.h.beta2 ** self.t
