"""Fault injection for the multi-process runtime.

A W = 3 gloo job on CPU (the same Trainer / exchange code that runs over RCCL on MI355X) in
which one rank dies mid-step (os._exit) or hangs (SIGSTOP).  The reference has no failure
handling at all: its PS blocks in ``comm.Recv`` forever on a dead worker
(``mnist_sync/parameter_server.py:57-69``).  Here every surviving rank must END with a
non-zero status within the watchdog bound — an error from the process group when the peer's
socket closes, or the step watchdog (``utils/watchdog.py``, ``Trainer._on_hang``: comm abort,
then ``os._exit(124)`` after at most ``ABORT_GRACE_S``) when the peer is alive but silent.
"""
import os
import signal
import subprocess
import sys
import time

import pytest

from conftest import ROOT, free_port

pytestmark = pytest.mark.slow

WATCHDOG_S = 6.0      # tests/fault_rank.py cpu config
GRACE_S = 5.0         # Trainer.ABORT_GRACE_S
SLACK_S = 25.0        # process start-up (import torch), set-up collectives, scheduling


def launch(tmp_path, world, device, fault, env_extra=None):
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    if device != "cpu":
        env = dict(os.environ, PYTHONPATH=ROOT)
    env.update(env_extra or {})
    procs = []
    for r in range(world):
        with open(os.path.join(tmp_path, f"rank{r}.log"), "w") as log:
            procs.append(subprocess.Popen(
                [sys.executable, os.path.join(ROOT, "tests", "fault_rank.py"), str(r), str(world),
                 str(port), device, fault, str(tmp_path)],
                env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True))
    return procs


def logs(tmp_path, world):
    return {r: open(os.path.join(tmp_path, f"rank{r}.log")).read()[-1500:] for r in range(world)}


def wait_survivors(procs, faulty, bound):
    """Exit codes of every rank but `faulty` (each must end within `bound` seconds of the
    first one that ends); the faulty rank is killed afterwards (a SIGSTOPped one never
    ends by itself)."""
    t0 = time.monotonic()
    codes = {}
    try:
        while len(codes) < len(procs) - 1:
            for r, p in enumerate(procs):
                if r != faulty and r not in codes and p.poll() is not None:
                    codes[r] = (p.returncode, time.monotonic() - t0)
            if time.monotonic() - t0 > bound:
                break
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        for p in procs:
            p.wait(timeout=30)
    return codes


@pytest.mark.parametrize("fault,faulty", [("kill@1:3", 1), ("stop@2:3", 2)])
def test_survivors_exit_nonzero_within_the_watchdog_bound(tmp_path, fault, faulty):
    world = 3
    procs = launch(tmp_path, world, "cpu", fault)
    bound = WATCHDOG_S + GRACE_S + SLACK_S + 60.0  # + first import of torch per process
    codes = wait_survivors(procs, faulty, bound)
    survivors = [r for r in range(world) if r != faulty]
    assert sorted(codes) == survivors, (f"survivors still running after {bound:.0f}s: {codes}",
                                        logs(tmp_path, world))
    for r, (rc, _) in codes.items():
        assert rc != 0, f"rank {r} exited 0 although rank {faulty} failed"
    # once the fault happened, the survivors ended close together: within one watchdog period
    # plus the abort grace of each other, not after a transport timeout of minutes
    ts = [t for _, t in codes.values()]
    assert max(ts) - min(ts) <= WATCHDOG_S + GRACE_S + 5.0, codes
    if fault.startswith("stop"):
        # a silent (stopped) peer is only detectable by the watchdog: status 124
        assert all(rc == 124 for rc, _ in codes.values()), codes
    assert procs[faulty].returncode != 0


def test_no_fault_completes_cleanly(tmp_path):
    """The harness itself: the same job without a fault ends with status 0 everywhere."""
    world = 2
    procs = launch(tmp_path, world, "cpu", "none", {"DDL_FAULT_STEPS": "4"})
    for p in procs:
        p.wait(timeout=600)
    assert [p.returncode for p in procs] == [0, 0], logs(tmp_path, world)
