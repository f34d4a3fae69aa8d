"""HIP engine: the CNN step on hand-written gfx950 kernels, replayed as HIP graphs.

The C++ ``Engine`` (``csrc/kernels/engine.hip``) owns all activation / gradient-scratch
buffers and launches every kernel of a step on torch's current stream.  This wrapper:

* binds the 14 parameter / gradient views of the plan-ordered flat buffers (so the
  exchange layer can slice PS shards straight out of them);
* keeps static input buffers (batch, labels, dropout seed as an int32 device word) so a
  step can be captured once and replayed;
* captures the forward + backward as **four HIP graphs**, one per backward segment
  (fc head, conv4, conv3, conv2+conv1); between replays it calls ``on_segment(s)`` so
  the sync exchange can push that segment's gradients on a side stream while the next
  graph computes.  A replay costs one host call instead of ~25 kernel launches.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from . import HIP_SEGMENTS
from .mnist_cnn import param_views
from ..ops import native


def _i32(seed: int) -> int:
    seed &= 0xFFFFFFFF
    return seed - (1 << 32) if seed >= (1 << 31) else seed


class HipEngine:
    name = "hip"
    segments = HIP_SEGMENTS

    def __init__(self, params: torch.Tensor, grads: torch.Tensor, offsets: Sequence[int],
                 batch: int = 100, graph: bool = True, eval_chunk: int = 10000,
                 keep_prob: float = 0.5, splits: Optional[List[int]] = None):
        if not params.is_cuda:
            raise ValueError("HipEngine needs GPU tensors")
        ext = native.ops()  # raises loudly if the extension is missing
        self.params, self.grads = params, grads
        self.pv = param_views(params, offsets)
        self.gv = param_views(grads, offsets)
        self.batch = batch
        # 10k rows = the reference's whole test set in one forward (7.25 ms vs 7.74 ms in 2k
        # chunks, scripts/eval_sweep.py); the activations for it take ~2.6 GB of 288 GB HBM
        self.eval_chunk = eval_chunk
        self.keep = keep_prob
        self.eng = ext.Engine([v.reshape(-1) for v in self.pv], [g.reshape(-1) for g in self.gv],
                              max(batch, eval_chunk), batch, keep_prob)
        if splits is not None:
            self.eng.set_splits(list(splits))
        dev = params.device
        self.x_static = torch.zeros(batch, 784, dtype=torch.float32, device=dev)
        self.y_static = torch.zeros(batch, dtype=torch.int64, device=dev)
        self.seed_static = torch.zeros(1, dtype=torch.int32, device=dev)
        self.use_graph = graph
        self.graphs: Optional[List[torch.cuda.CUDAGraph]] = None
        self._warm = False

    # ---- configuration ---------------------------------------------------------------------
    def set_splits(self, splits: List[int]) -> None:
        self.eng.set_splits(list(splits))
        self.graphs = None  # workspace was reallocated

    def get_splits(self) -> List[int]:
        return list(self.eng.get_splits())

    def set_cfg(self, cfg: List[int]) -> None:
        """Per-op block-tile configuration (see csrc/kernels/api.h NUM_TILE_CFGS)."""
        self.eng.set_cfg(list(cfg))
        self.graphs = None

    def get_cfg(self) -> List[int]:
        return list(self.eng.get_cfg())

    def set_wide(self, wide: List[int]) -> None:
        """Per-op split-K reduce threshold: splits > wide[op] use the separate wide-reduce
        kernel, otherwise the in-launch last-arriver reduction (csrc/kernels/gemm.h)."""
        self.eng.set_wide(list(wide))

    def get_wide(self) -> List[int]:
        return list(self.eng.get_wide())

    def set_concurrent(self, on: bool) -> None:
        """Weight-gradient GEMMs on a second stream (fork/join per backward segment)."""
        self.eng.set_concurrent(bool(on))
        self.graphs = None

    def set_dual(self, on: bool) -> None:
        """Single stream: each layer's data- and weight-gradient GEMMs in one launch."""
        self.eng.set_dual(bool(on))
        self.graphs = None

    def _set_keep(self, keep: float) -> None:
        if keep != self.keep:
            self.eng.set_keep_prob(keep)
            self.keep = keep
            self.graphs = None

    # ---- step ----------------------------------------------------------------------------------
    def _eager(self, x, y, seed_t, on_segment):
        self.eng.forward(x, seed_t, True)
        for s in range(len(self.segments)):
            self.eng.backward_segment(s, x, y, seed_t)
            if on_segment is not None:
                on_segment(s)

    def _capture(self) -> None:
        # warm up once eagerly (code-object load must not happen inside capture)
        torch.cuda.synchronize()
        graphs = []
        side = torch.cuda.Stream(device=self.params.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for s in range(len(self.segments)):
                g = torch.cuda.CUDAGraph()
                # thread_local: RCCL's watchdog thread keeps polling events while we capture
                with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                    if s == 0:
                        self.eng.forward(self.x_static, self.seed_static, True)
                    self.eng.backward_segment(s, self.x_static, self.y_static, self.seed_static)
                graphs.append(g)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graphs = graphs

    def forward_backward(self, x: torch.Tensor, labels: torch.Tensor, keep_prob: float, seed: int,
                         on_segment=None) -> None:
        self._set_keep(keep_prob)
        B = x.shape[0]
        if B != self.batch or not self.use_graph:
            if B > self.batch:
                raise ValueError(f"batch {B} > engine batch {self.batch}")
            # fill_ enqueues the value by argument: no host<->device sync, so the host keeps
            # running ahead of the GPU across steps (a torch.tensor(..., device=) H2D copy
            # here blocked the host every step until the GPU drained).
            self.seed_static.fill_(_i32(seed))
            self._eager(x.contiguous(), labels, self.seed_static, on_segment)
            return
        self.x_static.copy_(x)
        self.y_static.copy_(labels)
        self.seed_static.fill_(_i32(seed))
        if not self._warm:
            self._eager(self.x_static, self.y_static, self.seed_static, None)
            self._warm = True
        if self.graphs is None:
            self._capture()
        for s, g in enumerate(self.graphs):
            g.replay()
            if on_segment is not None:
                on_segment(s)

    def loss(self) -> torch.Tensor:
        return self.eng.buffer("loss", self.batch).mean()

    # ---- eval ------------------------------------------------------------------------------------
    @torch.no_grad()
    def correct_async(self, x: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        """Enqueue the correct-count eval on the current stream; returns the device int32
        [1] counter (valid once the stream reaches this point; no host sync)."""
        self.eng.zero_correct()
        for i in range(0, x.shape[0], self.eval_chunk):
            self.eng.eval_count(x[i:i + self.eval_chunk].contiguous(),
                                labels[i:i + self.eval_chunk].contiguous())
        return self.eng.buffer("correct", 1)

    @torch.no_grad()
    def correct(self, x: torch.Tensor, labels: torch.Tensor) -> int:
        return int(self.correct_async(x, labels).item())

    def accuracy(self, x: torch.Tensor, labels: torch.Tensor) -> float:
        return self.correct(x, labels) / x.shape[0]

    @torch.no_grad()
    def logits(self, x: torch.Tensor) -> torch.Tensor:
        """fp32 logits via the HIP forward (+ fc3 in torch; the fused head kernel only
        emits the loss / correct count)."""
        seed_t = torch.zeros(1, dtype=torch.int32, device=x.device)
        self.eng.forward(x.contiguous(), seed_t, False)
        h2 = self.eng.buffer("h2", x.shape[0])
        return h2 @ self.pv[12] + self.pv[13]
