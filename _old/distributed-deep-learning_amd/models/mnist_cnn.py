"""The reference MNIST CNN: parameter views, TF1 init, and the torch oracle engine.

Graph (``mnist_sync/model/model.py:17-92``), NHWC activations, HWIO weights:

    x[N,784] -> [N,28,28,1]
    4 x { conv5x5 SAME -> +b -> ReLU -> maxpool 2x2/2 SAME }   (28->14->7->4->2)
    flatten [N,1024] -> fc1 (+b, ReLU) -> dropout
                     -> fc2 (+b, *no* activation) -> dropout
                     -> fc3 (+b) = logits -> softmax cross-entropy (mean)

``TorchEngine`` is the plain-PyTorch implementation of those semantics.  It is the
CPU path (tests, gloo protocol rehearsal, ``single.py`` without a GPU) and, run on a
GPU with stock ops, the *faithful baseline* that ``bench.py --engine torch`` measures.
The production path is ``models/hip_engine.py`` (hand-written gfx950 kernels).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F

from .layout import TENSORS, NUM_CLASSES, CONV_LAYERS
from ..ops import rng

DROPOUT_LAYER_FC1 = 1
DROPOUT_LAYER_FC2 = 2


def glorot_limit(shape: Sequence[int]) -> float:
    """TF1 ``glorot_uniform`` limit; biases (rank 1) use fan_in = fan_out = n
    (``get_variable`` without an initializer) [TF-semantics]."""
    if len(shape) == 1:
        fan_in = fan_out = shape[0]
    elif len(shape) == 2:
        fan_in, fan_out = shape
    else:
        receptive = 1
        for s in shape[:-2]:
            receptive *= s
        fan_in, fan_out = shape[-2] * receptive, shape[-1] * receptive
    return math.sqrt(6.0 / (fan_in + fan_out))


def param_views(flat: torch.Tensor, offsets: Sequence[int]) -> List[torch.Tensor]:
    """Shaped views ``v0..v13`` into a flat buffer laid out by ``offsets``."""
    views = []
    for t in TENSORS:
        o = offsets[t.index]
        views.append(flat[o:o + t.numel].view(t.shape))
    return views


def init_params_(flat: torch.Tensor, offsets: Sequence[int], seed: int = 0) -> None:
    """Glorot-uniform init of every tensor (weights and biases), deterministic in ``seed``.

    Values are generated on the CPU in canonical order and copied in, so every rank and
    every device layout gets bit-identical parameters for the same seed."""
    gen = torch.Generator(device="cpu").manual_seed(int(seed))
    for t, view in zip(TENSORS, param_views(flat, offsets)):
        lim = glorot_limit(t.shape)
        vals = (torch.rand(t.shape, generator=gen, dtype=torch.float32) * 2.0 - 1.0) * lim
        view.copy_(vals)


def _pool_same(h: torch.Tensor) -> torch.Tensor:
    # NCHW max-pool 2x2/2 with TF SAME padding (pad bottom/right with -inf when odd).
    H = h.shape[-1]
    if H % 2:
        h = F.pad(h, (0, 1, 0, 1), value=float("-inf"))
    return F.max_pool2d(h, 2, 2)


def dropout_apply(h: torch.Tensor, seed: int, layer: int, keep_prob: float) -> torch.Tensor:
    if keep_prob >= 1.0:
        return h
    mask = rng.keep_mask(seed, layer, h.numel(), keep_prob, device=h.device).view_as(h)
    return torch.where(mask, h * (1.0 / keep_prob), torch.zeros_like(h))


def torch_forward(p: Sequence[torch.Tensor], x: torch.Tensor, keep_prob: float = 1.0,
                  seed: int = 0) -> torch.Tensor:
    """Logits [N,10] for flat images x [N,784]."""
    n = x.shape[0]
    h = x.view(n, 1, 28, 28)  # NHWC with C=1 == NCHW
    for li in range(len(CONV_LAYERS)):
        w, b = p[2 * li], p[2 * li + 1]
        h = F.conv2d(h, w.permute(3, 2, 0, 1), b, padding=2)
        h = _pool_same(F.relu(h))
    h = h.permute(0, 2, 3, 1).reshape(n, -1)  # TF flattens NHWC
    h = F.relu(h @ p[8] + p[9])
    h = dropout_apply(h, seed, DROPOUT_LAYER_FC1, keep_prob)
    h = h @ p[10] + p[11]
    h = dropout_apply(h, seed, DROPOUT_LAYER_FC2, keep_prob)
    return h @ p[12] + p[13]


def xent_loss(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """``reduce_mean(softmax_cross_entropy_with_logits)`` with integer labels."""
    return F.cross_entropy(logits, labels)


class TorchEngine:
    """Stock-PyTorch compute engine over a flat parameter buffer.

    ``params`` / ``grads`` are flat fp32 buffers laid out by ``offsets`` (a shard
    plan's plan-ordered layout), so the communication layer can slice PS shards
    directly out of them.
    """

    name = "torch"

    def __init__(self, params: torch.Tensor, grads: torch.Tensor, offsets: Sequence[int],
                 batch: int = 100):
        self.params, self.grads, self.offsets = params, grads, list(offsets)
        self.batch = batch
        self.pv = param_views(params, offsets)
        self.gv = param_views(grads, offsets)

    segments = [list(range(len(TENSORS)))]

    def forward_backward(self, x: torch.Tensor, labels: torch.Tensor, keep_prob: float,
                         seed: int, on_segment=None) -> torch.Tensor:
        leaves = [v.detach().requires_grad_(True) for v in self.pv]
        logits = torch_forward(leaves, x, keep_prob, seed)
        loss = xent_loss(logits, labels)
        gs = torch.autograd.grad(loss, leaves)
        with torch.no_grad():
            for dst, g in zip(self.gv, gs):
                dst.copy_(g)
        if on_segment is not None:
            on_segment(0)
        return loss.detach()

    @torch.no_grad()
    def logits(self, x: torch.Tensor) -> torch.Tensor:
        return torch_forward(self.pv, x, 1.0, 0)

    @torch.no_grad()
    def correct(self, x: torch.Tensor, labels: torch.Tensor, chunk: int = 2000) -> int:
        tot = 0
        for i in range(0, x.shape[0], chunk):
            lg = self.logits(x[i:i + chunk])
            tot += int((lg.argmax(1) == labels[i:i + chunk]).sum())
        return tot

    def accuracy(self, x: torch.Tensor, labels: torch.Tensor) -> float:
        return self.correct(x, labels) / x.shape[0]
