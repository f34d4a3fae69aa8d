"""Tracing: roctx ranges per phase (fwd/bwd, exchange, eval) + host step timers.

The reference's only timing is ``time.clock()``.  Ranges are emitted
through ``torch.cuda.nvtx`` which maps to roctx on ROCm, so ``rocprofv3 --marker-trace``
shows them next to the kernel trace.  Enable with ``DDL_TRACE=1``.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict

_ENABLED = os.environ.get("DDL_TRACE", "0") == "1"


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED:
        yield
        return
    import torch
    pushed = False
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


class StepTimer:
    """Accumulates wall time per named phase (host side)."""

    def __init__(self):
        self.tot = defaultdict(float)
        self.cnt = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.tot[name] += time.perf_counter() - t0
            self.cnt[name] += 1

    def summary(self):
        return {k: {"total_s": v, "count": self.cnt[k], "mean_ms": 1e3 * v / max(self.cnt[k], 1)}
                for k, v in self.tot.items()}
