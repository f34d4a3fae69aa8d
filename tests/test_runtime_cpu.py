"""Runtime pieces on CPU: native shm mailbox, store mailbox, checkpoint/resume, watchdog,
data loaders, reference print lines, entry scripts."""
import json
import multiprocessing as mp
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from conftest import ROOT, free_port
from ddl_amd.ops import native
from ddl_amd.parallel import mailbox as mbox
from ddl_amd.utils import metrics
from ddl_amd.utils.data import synthetic_mnist, load_file, batch_indices
from ddl_amd.utils.watchdog import Watchdog

needs_native = pytest.mark.skipif(not native.available(), reason="native extension not built")


def _producer(name, wid, n):
    sys.path.insert(0, ROOT)
    from ddl_amd.ops import native as nat
    mb = nat.ops().ShmMailbox(name, 64, False)
    for i in range(n):
        assert mb.push(mbox.encode(wid, i), 10.0)


@needs_native
def test_shm_mailbox_multiprocess_fifo_per_producer():
    name = f"/ddltest_{os.getpid()}"
    owner = native.ops().ShmMailbox(name, 64, True)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_producer, args=(name, w, 200)) for w in range(4)]
    for p in procs:
        p.start()
    got = {w: [] for w in range(4)}
    for _ in range(800):
        v = owner.pop(30.0)
        assert v >= 0
        w, i = mbox.decode(v)
        got[w].append(i)
    for p in procs:
        p.join()
        assert p.exitcode == 0
    assert owner.pop(0.05) == -1          # empty -> timeout sentinel
    for w in range(4):
        assert got[w] == list(range(200))  # per-producer order preserved, nothing lost
    owner.unlink()


@needs_native
def test_shm_mailbox_full_times_out():
    name = f"/ddltest_full_{os.getpid()}"
    mb = native.ops().ShmMailbox(name, 4, True)
    for i in range(mb.capacity()):
        assert mb.push(i, 1.0)
    t0 = time.time()
    assert not mb.push(99, 0.05)
    assert time.time() - t0 < 2.0
    assert mb.size() == mb.capacity()
    mb.unlink()


def test_store_mailbox_roundtrip():
    import torch.distributed as dist
    port = free_port()
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    a = mbox.StoreMailbox(store, "mb", True)
    b = mbox.StoreMailbox(store, "mb", False)
    for i in range(5):
        b.push(mbox.encode(1, i))
    assert [mbox.decode(a.pop(5.0)) for _ in range(5)] == [(1, i) for i in range(5)]
    assert a.pop(0.2) is None


def test_watchdog_fires_and_kick_prevents():
    fired = []
    wd = Watchdog(0.3, "t", on_timeout=lambda: fired.append(1))
    for _ in range(5):
        time.sleep(0.1)
        wd.kick()
    assert not fired
    time.sleep(1.5)
    assert fired and wd.fired
    wd.stop()


_BLOCKED_ABORT = r"""
import sys, threading, time
sys.path.insert(0, sys.argv[1])
from ddl_amd.parallel.roles import Trainer
class Ex:  # a communicator abort that never returns (e.g. stuck on a dead peer)
    def abort(self):
        threading.Event().wait()
t = Trainer.__new__(Trainer)
t.exchange = Ex()
Trainer.ABORT_GRACE_S = 0.5
t0 = time.monotonic()
t._on_hang()
"""


def test_watchdog_exits_even_if_comm_abort_blocks():
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", _BLOCKED_ABORT, ROOT], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 124, r.stderr
    assert "still blocked" in r.stderr
    assert time.monotonic() - t0 < 30


def test_synthetic_data_shapes_and_learnability():
    d = synthetic_mnist(2000, 500, seed=3)
    assert d.x_train.shape == (2000, 784) and d.y_train.shape == (2000,)
    assert d.x_test.shape == (500, 784)
    assert 0.0 <= float(d.x_train.min()) and float(d.x_train.max()) <= 1.0
    assert d.one_hot_train().shape == (2000, 10)
    # nearest-prototype classification is well above chance => learnable
    means = torch.stack([d.x_train[d.y_train == c].mean(0) for c in range(10)])
    pred = torch.cdist(d.x_test, means).argmin(1)
    assert (pred == d.y_test).float().mean() > 0.5


def test_npz_loader(tmp_path):
    f = tmp_path / "m.npz"
    np.savez(f, x_train=np.zeros((10, 784), np.float32), y_train=np.arange(10),
             x_test=np.ones((4, 784), np.float32), y_test=np.arange(4))
    d = load_file(str(f))
    assert d.x_train.shape == (10, 784) and int(d.y_test[3]) == 3


@pytest.mark.parametrize("gz", [False, True])
def test_reference_pickle_loads_arrays(tmp_path, gz):
    """The reference's mnist.pkl layout ((train, valid, test) tuples of numpy arrays, protocol 2
    as written by python 2 and the current protocol) loads through the array-only unpickler."""
    import gzip
    import pickle
    rng = np.random.default_rng(0)
    tr = (rng.random((6, 784), dtype=np.float32), np.arange(6, dtype=np.int64))
    va = (np.zeros((2, 784), np.float32), np.zeros(2, np.int64))
    te = (rng.random((3, 784), dtype=np.float32), np.array([7, 8, 9]))
    for proto in (2, pickle.HIGHEST_PROTOCOL):
        f = tmp_path / f"m{proto}.pkl{'.gz' if gz else ''}"
        with (gzip.open if gz else open)(f, "wb") as h:
            pickle.dump((tr, va, te), h, protocol=proto)
        d = load_file(str(f))
        assert torch.equal(d.x_train, torch.from_numpy(tr[0]))
        assert d.y_test.tolist() == [7, 8, 9]


class _Evil:
    def __reduce__(self):
        import os
        return (os.system, ("echo pwned",))


def test_reference_pickle_refuses_other_globals(tmp_path):
    """A pickle carrying any global but the numpy array reconstructors is refused before
    anything it names is called."""
    import pickle
    arr = (np.zeros((1, 784), np.float32), np.zeros(1, np.int64))
    for payload in [(arr, arr, (_Evil(), arr[1])), (arr, arr, (arr[0], [print]))]:
        f = tmp_path / "evil.pkl"
        f.write_bytes(pickle.dumps(payload))
        with pytest.raises(pickle.UnpicklingError, match="refusing global"):
            load_file(str(f))


def test_shared_gpu_ranks_get_one_hw_queue(monkeypatch):
    from ddl_amd.parallel import comm
    monkeypatch.delenv("DDL_SHARED_GPU_HW_QUEUES", raising=False)
    monkeypatch.delenv("DDL_COMM_PRIORITY", raising=False)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")          # what the GPU boxes export
    monkeypatch.setattr(comm.torch.cuda, "device_count", lambda: 1)
    assert comm.share_gpu_queue_cap(1) is None           # one process: HIP's default
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"
    assert comm.share_gpu_queue_cap(4) == "1"             # four ranks on one card
    assert os.environ["GPU_MAX_HW_QUEUES"] == "1"
    assert os.environ["DDL_COMM_PRIORITY"] == "low"        # and the comm stream at low priority
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setenv("DDL_SHARED_GPU_HW_QUEUES", "keep")
    assert comm.share_gpu_queue_cap(4) is None and os.environ["GPU_MAX_HW_QUEUES"] == "4"
    monkeypatch.setenv("DDL_SHARED_GPU_HW_QUEUES", "2")
    assert comm.share_gpu_queue_cap(4) == "2" and os.environ["GPU_MAX_HW_QUEUES"] == "2"
    monkeypatch.delenv("DDL_SHARED_GPU_HW_QUEUES")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setattr(comm.torch.cuda, "device_count", lambda: 8)
    assert comm.share_gpu_queue_cap(8) is None            # one process per GPU
    monkeypatch.setattr(comm.torch.cuda, "device_count", lambda: 0)
    assert comm.share_gpu_queue_cap(4) is None            # CPU ranks


def test_batch_indices_semantics():
    # reference: every worker walks the same slices (Q5)
    assert batch_indices(3, 100, 50000, rank=2, world=4) == (300, 400)
    assert batch_indices(3, 100, 50000, rank=2, world=4, sharding="stride") == (1400, 1500)
    assert batch_indices(500, 100, 50000) == (0, 100)  # wraps after one epoch


def test_reference_print_lines():
    assert metrics.worker_progress(1, 0, 10, 0.5) == "Worker1 epoch: 0 batch: 10 accuracy: 0.5"
    assert metrics.worker_final(1, 0.9) == "Worker1 final accuracy: 0.9"
    assert metrics.single_progress(0, 10, 0.5) == "epoch: 0 batch: 10 accuracy: 0.5"
    assert metrics.single_final(0.9) == "final accuracy: 0.9"
    assert metrics.time_line(1.5) == "Time: 1.5"


def _trainer(tmp, shard="contiguous", num_ps=None, steps=3):
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    cfg = TrainConfig(mode="sync", shard=shard, num_ps=num_ps, steps=steps, batch_size=20,
                      eval_every=0, quiet=True, engine="torch", checkpoint_dir=str(tmp))
    return Trainer(cfg, DistEnv(), dataset=synthetic_mnist(200, 50, seed=1))


def test_checkpoint_roundtrip_and_reshard(tmp_path):
    from safetensors.torch import load_file as st_load
    tr = _trainer(tmp_path, "contiguous", 3)
    tr.train()
    man = json.load(open(tmp_path / "manifest.json"))
    assert man["global_step"] == 3 and man["ps_t"] == {"0": 3, "1": 3, "2": 3}
    w = st_load(str(tmp_path / "worker0.safetensors"))
    assert sorted(w) == sorted(f"mnist/v{i}" for i in range(14))
    ps0 = st_load(str(tmp_path / "ps0.safetensors"))
    assert "ParameterServer/v0/Adam" in ps0 and "ParameterServer/v0/Adam_1" in ps0
    assert "ParameterServer/beta1_power" in ps0
    assert float(ps0["ParameterServer/beta1_power"][0]) == pytest.approx(0.9 ** 3)
    # resume into a *different* plan (flat, 2 PS): parameters and Adam slots carry over
    from ddl_amd.utils import checkpoint as ckpt
    tr2 = _trainer(tmp_path / "other", "flat", 2)
    ckpt.load(tr2, str(tmp_path))
    from ddl_amd.models.layout import TENSORS
    for t in TENSORS:
        a = tr.params[tr.plan.tensor_offsets[t.index]:][:t.numel]
        b = tr2.params[tr2.plan.tensor_offsets[t.index]:][:t.numel]
        assert torch.equal(a, b)
    # Adam m of v8 from PS that owned it
    owner = tr.plan.owner[8]
    o_old = tr.plan.tensor_offsets[8] - tr.plan.ps_ranges[owner][0]
    m_old = tr.servers[owner].m[o_old:o_old + 10]
    o_new = tr2.plan.tensor_offsets[8]
    found = False
    for ps in tr2.servers.values():
        for (lo, hi), off in zip(ps.segments, ps.seg_off):
            if lo <= o_new < hi:
                s = off + o_new - lo
                assert torch.equal(ps.m[s:s + 10], m_old)
                found = True
    assert found
    assert all(ps.t == 3 for ps in tr2.servers.values()) and tr2.global_step == 3


def test_single_py_cli_prints_reference_lines():
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "single.py", "--steps", "11", "--data", "synthetic:1000",
                        "--batch-size", "20"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert lines[0].startswith("epoch: 0 batch: 0 accuracy: ")
    assert lines[1].startswith("epoch: 0 batch: 10 accuracy: ")
    assert lines[2].startswith("final accuracy: ")
    assert lines[3].startswith("Time: ")


def test_run_sh_launches_two_workers():
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               MASTER_PORT=str(free_port()))
    r = subprocess.run(["bash", "run.sh", "2", "2", "--variant", "mnist_sync_sharding_greedy",
                        "--steps", "2", "--data", "synthetic:600", "--batch-size", "20",
                        "--eval-every", "0"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Worker0 final accuracy:" in r.stdout and "Worker1 final accuracy:" in r.stdout


def test_eval_async_without_hip_engine_falls_back_to_inline_eval():
    """--eval-async needs the HIP engine; on the CPU torch engine the reference in-line eval
    runs and gives the same history."""
    import torch
    from ddl_amd.config import TrainConfig
    from ddl_amd.parallel.comm import DistEnv
    from ddl_amd.parallel.roles import Trainer
    from ddl_amd.utils.data import synthetic_mnist
    data = synthetic_mnist(n_train=400, n_test=200, seed=3)
    hist = []
    for ea in (False, True):
        cfg = TrainConfig(mode="single", shard="none", steps=4, batch_size=50, eval_every=2,
                          engine="torch", quiet=True, eval_async=ea)
        tr = Trainer(cfg, DistEnv(device=torch.device("cpu")), dataset=data)
        tr.train()
        hist.append([(h["step"], h["acc"]) for h in tr.history])
    assert len(hist[0]) == 2 and hist[0] == hist[1]


def test_exchange_flag_and_cpu_fallback():
    """--exchange reaches the config; on a CPU (no HIP engine) the native runner is not
    available, so the sync exchange falls back to the Python one whatever the flag says."""
    import argparse
    from ddl_amd.config import add_args, from_args, TrainConfig
    from ddl_amd.parallel.comm import DistEnv, SyncExchange
    from ddl_amd.parallel.roles import Trainer
    a = add_args(argparse.ArgumentParser()).parse_args(["--exchange", "xgmi", "--shard", "flat"])
    cfg = from_args(a)
    assert cfg.exchange_backend == "xgmi"
    cfg = TrainConfig(mode="sync", shard="flat", steps=1, batch_size=20, eval_every=0,
                      quiet=True, engine="torch", exchange_backend="xgmi")
    tr = Trainer(cfg, DistEnv(), dataset=synthetic_mnist(200, 50, seed=1))
    assert type(tr.exchange) is SyncExchange and not getattr(tr.exchange, "native", False)
    tr.train_step(0)
