"""CPU numerics: dropout RNG, TF1 Adam, glorot init, model oracle, quirk coefficients."""
import math

import pytest
import torch

from ddl_amd.models.layout import TENSORS, CANON_OFFSETS, TOTAL_NUMEL, forward_flops_per_sample
from ddl_amd.models.mnist_cnn import (glorot_limit, init_params_, param_views, torch_forward,
                                      xent_loss, TorchEngine, _pool_same)
from ddl_amd.ops import rng
from ddl_amd.ops.adam import AdamHyper, adam_torch_, adam_coeffs
from ddl_amd.parallel.comm import quirk_coefficient
from ddl_amd.parallel.sharding import make_plan
from ddl_amd.parallel.ps import ParameterServer


def test_forward_flops_constant():
    # 70.77 MFLOP / sample
    assert forward_flops_per_sample() / 1e6 == pytest.approx(70.77, abs=0.01)


def test_dropout_mask_rate_and_determinism():
    m1 = rng.keep_mask(123, 1, 200000, 0.5)
    m2 = rng.keep_mask(123, 1, 200000, 0.5)
    assert torch.equal(m1, m2)
    assert abs(m1.float().mean().item() - 0.5) < 0.01
    m3 = rng.keep_mask(124, 1, 200000, 0.5)
    assert not torch.equal(m1, m3)
    assert rng.keep_mask(1, 1, 100, 1.0).all()
    assert abs(rng.keep_mask(9, 2, 200000, 0.8).float().mean().item() - 0.8) < 0.01


def test_mix_scalar_matches_tensor():
    xs = [0, 1, 12345, 0xFFFFFFFF, 0x9E3779B9]
    t = rng._mix(torch.tensor(xs, dtype=torch.int64))
    assert [rng.mix_scalar(x) for x in xs] == t.tolist()


def test_glorot_limits():
    assert glorot_limit((5, 5, 1, 32)) == pytest.approx(math.sqrt(6 / (25 + 800)))
    assert glorot_limit((1024, 512)) == pytest.approx(math.sqrt(6 / 1536))
    assert glorot_limit((32,)) == pytest.approx(math.sqrt(3 / 32))  # biases too (§2.5)


def test_init_within_limits_and_deterministic():
    a = torch.zeros(TOTAL_NUMEL)
    b = torch.zeros(TOTAL_NUMEL)
    init_params_(a, CANON_OFFSETS, 5)
    init_params_(b, CANON_OFFSETS, 5)
    assert torch.equal(a, b)
    for t, v in zip(TENSORS, param_views(a, CANON_OFFSETS)):
        assert v.abs().max() <= glorot_limit(t.shape) + 1e-7


def test_same_pool_pads_bottom_right():
    h = torch.arange(49.0).view(1, 1, 7, 7) - 100  # all negative -> -inf pad must not win
    p = _pool_same(h)
    assert p.shape == (1, 1, 4, 4)
    assert p[0, 0, 3, 3] == h[0, 0, 6, 6]


def test_tf1_adam_matches_closed_form():
    h = AdamHyper()
    w = torch.tensor([1.0, -2.0])
    m = torch.zeros(2)
    v = torch.zeros(2)
    g = torch.tensor([0.5, -0.25])
    adam_torch_(w, g, m, v, h, 1)
    # step 1: m = 0.1 g, v = 0.001 g^2, lr_t = lr * sqrt(1-b2)/(1-b1)
    lr_t = 1e-4 * math.sqrt(0.001) / 0.1
    exp = torch.tensor([1.0, -2.0]) - lr_t * (0.1 * g) / ((0.001 * g * g).sqrt() + 1e-8)
    assert torch.allclose(w, exp, atol=1e-9)
    assert adam_coeffs(h, 1) == pytest.approx(lr_t)


def test_ps_step_counter_per_server():
    plan = make_plan("contiguous", 2)
    ps0 = ParameterServer(plan, 0, "cpu")
    ps1 = ParameterServer(plan, 1, "cpu")
    w = torch.zeros(plan.total)
    g = torch.ones(plan.total)
    ps0.update_flat(w, g)
    ps0.update_flat(w, g)
    ps1.update_flat(w, g)
    assert (ps0.t, ps1.t) == (2, 1)
    lo0, hi0 = plan.ps_ranges[0]
    lo1, hi1 = plan.ps_ranges[1]
    # Adam's first steps move every weight by ~lr regardless of |g|
    assert w[lo0:hi0].mean().item() == pytest.approx(-2e-4, rel=1e-3)
    assert w[lo1:hi1].mean().item() == pytest.approx(-1e-4, rel=1e-3)


def test_quirk_goldens():
    # W=3, g=(1,2,3): Q1 -> 7, Q2 -> 12
    g = [1.0, 2.0, 3.0]
    none = make_plan("none", 1)
    shard = make_plan("contiguous", 3)
    assert sum(quirk_coefficient(none, r, 3, True) * g[r] for r in range(3)) == 7
    assert sum(quirk_coefficient(shard, r, 3, True) * g[r] for r in range(3)) == 12
    assert sum(quirk_coefficient(shard, r, 3, False) * g[r] for r in range(3)) == 6


def test_torch_engine_grads_match_finite_difference():
    torch.manual_seed(0)
    flat = torch.zeros(TOTAL_NUMEL, dtype=torch.float64)
    init_params_(flat, CANON_OFFSETS, 1)
    grads = torch.zeros_like(flat)
    eng = TorchEngine(flat, grads, CANON_OFFSETS, batch=4)
    x = torch.rand(4, 784, dtype=torch.float64)
    y = torch.tensor([1, 3, 5, 7])
    eng.forward_backward(x, y, 1.0, 0)
    pv = param_views(flat, CANON_OFFSETS)
    for ti, idx in [(13, 3), (8, 5), (0, 7), (11, 2)]:
        v = pv[ti].view(-1)
        old = v[idx].item()
        eps = 1e-6
        v[idx] = old + eps
        lp = xent_loss(torch_forward(pv, x, 1.0, 0), y).item()
        v[idx] = old - eps
        lm = xent_loss(torch_forward(pv, x, 1.0, 0), y).item()
        v[idx] = old
        fd = (lp - lm) / (2 * eps)
        an = param_views(grads, CANON_OFFSETS)[ti].view(-1)[idx].item()
        assert an == pytest.approx(fd, rel=1e-4, abs=1e-9)


def test_fc2_has_no_activation():
    # Q10: negative pre-activations of fc2 must pass through (times dropout scale)
    flat = torch.zeros(TOTAL_NUMEL)
    pv = param_views(flat, CANON_OFFSETS)
    pv[11].fill_(-1.0)       # fc2 bias
    pv[12].copy_(torch.eye(512, 10))
    out = torch_forward(pv, torch.zeros(2, 784), 1.0, 0)
    assert torch.allclose(out, torch.full((2, 10), -1.0))
