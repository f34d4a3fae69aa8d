"""The C++ SyncRunner (csrc/kernels/runner.hip) vs the Python SyncExchange on one GPU.

Both enqueue the same HIP kernels on the same plan ranges, so after several steps the
parameters, the Adam moments and the PS step counters must be bit-identical — for every
shard policy (units with one / several PS, several ranges per unit, bucketed flat plan),
with and without overlap, for Adam and momentum.
"""
import pytest
import torch

from ddl_amd.config import TrainConfig
from ddl_amd.parallel.comm import DistEnv
from ddl_amd.parallel.roles import Trainer
from ddl_amd.utils.data import synthetic_mnist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data():
    return synthetic_mnist(n_train=2000, n_test=500, seed=5)


def _run(data, native, steps=6, **kw):
    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", steps=steps, batch_size=100, eval_every=0, engine="hip",
                      quiet=True, native_exchange=native, **kw)
    tr = Trainer(cfg, env, dataset=data)
    assert getattr(tr.exchange, "native", False) == native
    for i in range(steps):
        tr.train_step(i)
    torch.cuda.synchronize()
    state = {p: (s.t, s.m.clone(), None if s.v is None else s.v.clone())
             for p, s in tr.servers.items()}
    return tr.params.clone(), state


@pytest.mark.parametrize("kw", [
    dict(shard="contiguous"),
    dict(shard="greedy", num_ps=3),
    dict(shard="contiguous", num_ps=2, overlap=False),
    dict(shard="flat"),
    dict(shard="lpt", num_ps=4, optimizer="momentum"),
])
def test_native_matches_python_exchange(data, kw):
    p_py, s_py = _run(data, False, **kw)
    p_nat, s_nat = _run(data, True, **kw)
    assert torch.equal(p_py, p_nat)
    assert s_py.keys() == s_nat.keys()
    for p in s_py:
        assert s_py[p][0] == s_nat[p][0]
        assert torch.equal(s_py[p][1], s_nat[p][1])
        if s_py[p][2] is not None:
            assert torch.equal(s_py[p][2], s_nat[p][2])


def test_native_runner_trains(data):
    env = DistEnv(0, 1, 0, torch.device("cuda", 0))
    cfg = TrainConfig(mode="sync", shard="contiguous", steps=60, batch_size=100, eval_every=0,
                      engine="hip", quiet=True, lr=1e-3)
    tr = Trainer(cfg, env, dataset=data)
    acc0 = tr.evaluate()
    for i in range(60):
        tr.train_step(i)
    assert tr.evaluate() > max(0.5, acc0 + 0.2)
