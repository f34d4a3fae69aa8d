"""Parameter-server shard state and update.

Reference PS (``mnist_sync_sharding/parameter_server.py:6-82``): owns a slice of the
14 variables under scope ``ParameterServer/v{i}``, an ``AdamOptimizer(1e-4)`` whose slots
(``Adam``/``Adam_1``) and ``beta1_power``/``beta2_power`` live in that PS's own graph,
sums incoming worker gradients with NumPy and runs ``apply_gradients``.

Here a PS is *co-located* in the process of the GPU that hosts it: its
shard is one or more element ranges of the plan-ordered flat buffer.  The update is the
fused ``adam_flat`` HIP kernel on those ranges (no host round trip, no per-tensor ops).
In sync mode the PS updates the host worker's own parameter buffer in place and the
result is broadcast/all-gathered; in async mode the PS keeps a private parameter copy
(``own_params``), because the host's worker thread keeps computing on its own copy.
"""
from __future__ import annotations

import contextlib
import threading
from typing import List, Optional, Tuple

import torch

from .sharding import ShardPlan
from ..ops import native
from ..ops.adam import AdamHyper, adam_coeffs


class ParameterServer:
    def __init__(self, plan: ShardPlan, ps_id: int, device, hyper: Optional[AdamHyper] = None,
                 optimizer: str = "adam", momentum: float = 0.9,
                 own_params: Optional[torch.Tensor] = None, native_optim: bool = True):
        self.plan, self.id, self.device = plan, ps_id, torch.device(device)
        # False only for the stock-PyTorch baseline engine (bench.py --engine torch)
        self.native_optim = native_optim
        self.h = hyper or AdamHyper()
        self.optimizer, self.momentum = optimizer, momentum
        self.segments: List[Tuple[int, int]] = plan.ps_segments(ps_id)
        self.seg_off: List[int] = []
        off = 0
        for lo, hi in self.segments:
            self.seg_off.append(off)
            off += hi - lo
        self.numel = off
        z = lambda: torch.zeros(self.numel, dtype=torch.float32, device=self.device)  # noqa: E731
        self.m = z()
        self.v = z() if optimizer == "adam" else None
        self.t = 0                       # this PS's own step counter (beta powers)
        self.updates = 0
        self.lock = threading.Lock()     # async: worker thread + service thread
        # async mode: private copy of the owned parameters, contiguous [numel]
        self.params = None
        if own_params is not None:
            self.params = torch.cat([own_params[lo:hi] for lo, hi in self.segments]).to(self.device)
        self.gbuf = None                 # receive buffer for remote gradients (async)
        # async: all updates of this PS are serialised on one stream under `lock` (created on
        # first use: sync runs never need it, and every HIP stream competes for the few
        # hardware queues)
        self._stream = None

    @property
    def stream(self):
        if self._stream is None and self.device.type == "cuda":
            self._stream = torch.cuda.Stream(device=self.device)
        return self._stream

    @contextlib.contextmanager
    def exclusive(self):
        """Lock the PS and run the body on its stream, ordered after the caller's stream
        on entry and before it on exit (host lock alone does not order GPU streams)."""
        with self.lock:
            if self.stream is None:
                yield
                return
            cur = torch.cuda.current_stream(self.device)
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                yield
            cur.wait_stream(self.stream)

    # ---- update --------------------------------------------------------------------------
    def begin(self) -> None:
        """One ``apply_gradients`` call: advance the step counter."""
        self.t += 1
        self.updates += 1

    def apply(self, w: torch.Tensor, g: torch.Tensor, state_off: int, grad_scale: float = 1.0) -> None:
        """Update the contiguous parameter view ``w`` from gradient view ``g``; Adam state
        at ``[state_off, state_off + w.numel())``."""
        n = w.numel()
        m = self.m[state_off:state_off + n]
        if self.optimizer == "adam":
            v = self.v[state_off:state_off + n]
            lr_t = adam_coeffs(self.h, self.t)
            if w.is_cuda and self.native_optim:
                native.ops().adam_flat(w, g, m, v, lr_t, self.h.beta1, self.h.beta2, self.h.eps,
                                       grad_scale)
            else:
                gg = g * grad_scale if grad_scale != 1.0 else g
                # TF ApplyAdam update form (same as the HIP kernel)
                m.add_((gg - m) * (1.0 - self.h.beta1))
                v.add_((gg * gg - v) * (1.0 - self.h.beta2))
                w.sub_(lr_t * m / (v.sqrt() + self.h.eps))
        elif self.optimizer == "momentum":
            if w.is_cuda and self.native_optim:
                native.ops().momentum_flat(w, g, m, self.h.lr, self.momentum, grad_scale)
            else:
                m.mul_(self.momentum).add_(g, alpha=grad_scale)
                w.sub_(self.h.lr * m)
        elif self.optimizer == "sgd":
            if w.is_cuda and self.native_optim:
                # the fused momentum kernel with mu = 0: w -= lr * (g * scale)
                native.ops().momentum_flat(w, g, m, self.h.lr, 0.0, grad_scale)
            else:
                w.sub_(g * grad_scale if grad_scale != 1.0 else g, alpha=self.h.lr)
        else:
            raise ValueError(self.optimizer)

    def update_flat(self, params: torch.Tensor, grads: torch.Tensor, grad_scale: float = 1.0) -> None:
        """Full-shard update in place on plan-ordered flat buffers (sync, local)."""
        self.begin()
        for (lo, hi), off in zip(self.segments, self.seg_off):
            self.apply(params[lo:hi], grads[lo:hi], off, grad_scale)

    def update_own(self, g_shard: torch.Tensor, grad_scale: float = 1.0) -> None:
        """Async: update the private copy from a packed shard gradient [numel]."""
        self.begin()
        self.apply(self.params, g_shard, 0, grad_scale)

    # ---- pack / unpack helpers (async) -----------------------------------------------------
    def gather_from(self, flat: torch.Tensor) -> torch.Tensor:
        if len(self.segments) == 1:
            lo, hi = self.segments[0]
            return flat[lo:hi]
        return torch.cat([flat[lo:hi] for lo, hi in self.segments])

    def scatter_to(self, flat: torch.Tensor, packed: torch.Tensor) -> None:
        for (lo, hi), off in zip(self.segments, self.seg_off):
            flat[lo:hi].copy_(packed[off:off + hi - lo])

    # ---- checkpoint ---------------------------------------------------------------------------
    def state_dict(self):
        d = {"t": self.t, "m": self.m}
        if self.v is not None:
            d["v"] = self.v
        if self.params is not None:
            d["params"] = self.params
        return d

    def load_state_dict(self, d):
        self.t = int(d["t"])
        self.m.copy_(d["m"])
        if self.v is not None and "v" in d:
            self.v.copy_(d["v"])
        if self.params is not None and "params" in d:
            self.params.copy_(d["params"])
