"""Arrival mailbox for the asynchronous parameter server.

The reference async PS receives with ``MPI.ANY_SOURCE`` and replies to whoever sent the
last tag (``mnist_async_sharding/parameter_server.py:99-111``).  RCCL has no wildcard
receive and every communicator needs a consistent op order (SURVEY.md §7.3 hard part 1),
so the wildcard becomes two pieces:

  1. a per-host arrival queue: a worker posts ``(worker, ps)`` *before* sending its
     gradient shard; the PS service thread pops entries in arrival order;
  2. a dedicated 2-rank communicator per (worker, PS host) pair for the data itself.

Two implementations:
  * ``ShmMailbox`` — native C++ lock-free bounded MPMC ring in POSIX shared memory
    (``csrc/runtime/mailbox.cpp``); one node, no syscalls on the fast path.
  * ``StoreMailbox`` — torch ``Store`` ticket counter (works across nodes, and when the
    native extension is not built).
"""
from __future__ import annotations

import datetime
import time
from typing import Optional

from ..ops import native


def encode(worker: int, ps: int) -> int:
    return (worker << 20) | ps


def decode(v: int):
    return v >> 20, v & ((1 << 20) - 1)


def _private_store(store):
    """A TCPStore client on its own connection: a blocking ``wait`` in the PS service
    thread must not serialise the worker thread's pushes behind it."""
    import os
    import torch.distributed as dist
    addr, port = os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")
    if addr and port:
        try:
            return dist.TCPStore(addr, int(port), is_master=False,
                                 timeout=datetime.timedelta(seconds=900))
        except Exception:
            pass
    return store


class StoreMailbox:
    def __init__(self, store, name: str, owner: bool):
        self.store, self.name = _private_store(store), name
        self.next = 0

    def push(self, value: int) -> None:
        ticket = self.store.add(f"{self.name}/tail", 1) - 1
        self.store.set(f"{self.name}/{ticket}", str(value))

    def pop(self, timeout_s: float = 600.0) -> Optional[int]:
        key = f"{self.name}/{self.next}"
        try:
            self.store.wait([key], datetime.timedelta(seconds=timeout_s))
        except Exception:
            return None
        v = int(self.store.get(key))
        self.store.delete_key(key)
        self.next += 1
        return v

    def close(self):
        pass


class ShmMailbox:
    def __init__(self, name: str, owner: bool, capacity: int = 4096):
        self.mb = native.ops().ShmMailbox(name, capacity, owner)
        self.owner = owner
        self.name = name

    def push(self, value: int) -> None:
        if not self.mb.push(value, 600.0):
            raise TimeoutError("mailbox full")

    def pop(self, timeout_s: float = 600.0) -> Optional[int]:
        v = self.mb.pop(timeout_s)
        return None if v < 0 else v

    def close(self):
        if self.owner:
            self.mb.unlink()


def make_mailbox(kind: str, store, name: str, owner: bool):
    if kind == "auto":
        kind = "shm" if native.available() and hasattr(native.ops(), "ShmMailbox") else "store"
    if kind == "shm":
        return ShmMailbox("/" + name.replace("/", "_"), owner)
    return StoreMailbox(store, name, owner)
