"""Failure detection: a per-process step watchdog.

The reference has none — any rank failure hangs ``mpiexec``.  Here each
training process runs a daemon thread that aborts the process (so torchrun tears the job
down and RCCL communicators are not left waiting forever) when no step completes within
``timeout_s``.  RCCL's own async error handling is enabled via
``TORCH_NCCL_ASYNC_ERROR_HANDLING`` in the launcher.
"""
from __future__ import annotations

import os
import sys
import threading
import time


class Watchdog:
    def __init__(self, timeout_s: float, name: str = "", on_timeout=None):
        self.timeout_s = float(timeout_s)
        self.name = name
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._stop = threading.Event()
        self.fired = False
        self._t = None
        if self.timeout_s > 0:
            self._t = threading.Thread(target=self._run, name="ddl-watchdog", daemon=True)
            self._t.start()

    def kick(self) -> None:
        self._last = time.monotonic()

    def _run(self) -> None:
        period = min(5.0, max(self.timeout_s / 4, 0.01))
        while not self._stop.wait(period):
            if time.monotonic() - self._last > self.timeout_s:
                self.fired = True
                msg = f"[watchdog {self.name}] no progress for {self.timeout_s:.1f}s - aborting\n"
                sys.stderr.write(msg)
                sys.stderr.flush()
                if self.on_timeout is not None:
                    self.on_timeout()
                    return
                os._exit(124)

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=1.0)
