"""Progress output: the reference's exact print lines plus structured JSONL.

Reference lines:
  worker  ``Worker{} epoch: {} batch: {} accuracy: {}``  (``mnist_sync/worker.py:72``)
          ``Worker{} final accuracy: {}``                 (``:75``)
          ``Time: {}``                                    (``:76``, CPU seconds)
  single  ``epoch: {} batch: {} accuracy: {}``            (``mnist_sync/single.py:18``)
          ``final accuracy: {}``                          (``:21``)
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Any, Dict, Optional


def worker_progress(rank: int, epoch: int, batch: int, acc: float) -> str:
    return "Worker{} epoch: {} batch: {} accuracy: {}".format(rank, epoch, batch, acc)


def worker_final(rank: int, acc: float) -> str:
    return "Worker{} final accuracy: {}".format(rank, acc)


def single_progress(epoch: int, batch: int, acc: float) -> str:
    return "epoch: {} batch: {} accuracy: {}".format(epoch, batch, acc)


def single_final(acc: float) -> str:
    return "final accuracy: {}".format(acc)


def time_line(seconds: float) -> str:
    return "Time: {}".format(seconds)


class Clock:
    """Wall clock and process CPU clock.  The reference's ``Time`` is CPU seconds from
    ``time.clock()`` (Python <= 3.7) — we report both."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.w0 = time.perf_counter()
        self.c0 = time.process_time()

    def wall(self) -> float:
        return time.perf_counter() - self.w0

    def cpu(self) -> float:
        return time.process_time() - self.c0


class JsonlLogger:
    def __init__(self, path: Optional[str] = None, rank: int = 0):
        self.rank = rank
        self.f = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
            self.f = open(path, "a")

    def log(self, **rec: Any) -> None:
        if self.f is None:
            return
        rec.setdefault("ts", time.time())
        rec.setdefault("rank", self.rank)
        self.f.write(json.dumps(rec) + "\n")
        self.f.flush()

    def close(self):
        if self.f:
            self.f.close()
            self.f = None


def emit(line: str) -> None:
    sys.stdout.write(line + "\n")
    sys.stdout.flush()
