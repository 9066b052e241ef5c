"""Flat fused optimizers vs torch.optim, clipping, LR schedules, FlatParams plumbing."""
import math

import pytest
import torch

import pcmp
from pcmp import optim as popt
from pcmp.utils.flat import FlatParams


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))


def _run(mine_cls, ref_cls, mkw, rkw, steps=5, clip=None):
    m1, m2 = _model(), _model()
    flat = FlatParams(m1.parameters(), shadow_dtype=None)
    o1 = mine_cls(flat, **mkw)
    o2 = ref_cls(m2.parameters(), **rkw)
    x, y = torch.randn(32, 8), torch.randint(0, 3, (32,))
    for _ in range(steps):
        o1.zero_grad()
        torch.nn.functional.cross_entropy(m1(x), y).backward()
        if clip:
            o1.clip_grad_norm(clip)
        o1.step()
        o2.zero_grad()
        torch.nn.functional.cross_entropy(m2(x), y).backward()
        if clip:
            torch.nn.utils.clip_grad_norm_(m2.parameters(), clip)
        o2.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-4)


def test_sgd_momentum_nesterov_wd():
    _run(popt.SGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True),
         dict(lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True))


def test_sgd_plain():
    _run(popt.SGD, torch.optim.SGD, dict(lr=0.05), dict(lr=0.05))


def test_adam():
    _run(popt.Adam, torch.optim.Adam, dict(lr=3e-3, weight_decay=1e-2), dict(lr=3e-3, weight_decay=1e-2))


def test_adamw_with_clip():
    _run(popt.AdamW, torch.optim.AdamW, dict(lr=2e-3, eps=1e-8, weight_decay=0.01),
         dict(lr=2e-3, eps=1e-8, weight_decay=0.01), clip=0.05)


def test_linear_schedule_matches_transformers():
    transformers = pytest.importorskip("transformers")
    m = _model()
    flat = FlatParams(m.parameters(), shadow_dtype=None)
    o = popt.AdamW(flat, lr=2e-5)
    s = popt.linear_schedule_with_warmup(o, 3, 20)
    m2 = _model()
    o2 = torch.optim.AdamW(m2.parameters(), lr=2e-5)
    s2 = transformers.get_linear_schedule_with_warmup(o2, 3, 20)
    for _ in range(22):
        assert math.isclose(o.lr, o2.param_groups[0]["lr"], rel_tol=1e-9, abs_tol=1e-15)
        o2.step()
        s.step()
        s2.step()


def test_flatparams_views_and_grad_fold():
    m = _model()
    before = [p.detach().clone() for p in m.parameters()]
    flat = FlatParams(m.parameters(), shadow_dtype=None)
    for p, b in zip(m.parameters(), before):
        assert torch.equal(p, b)
        assert p.data_ptr() >= flat.master.data_ptr()
    # torch-native autograd grads are folded into main_grad and p.grad cleared
    torch.nn.functional.cross_entropy(m(torch.randn(4, 8)), torch.tensor([0, 1, 2, 0])).backward()
    assert all(p.grad is None for p in m.parameters())
    assert flat.grad.abs().sum() > 0
    flat.zero_grad()
    torch.nn.functional.cross_entropy(m(torch.randn(4, 8)), torch.tensor([0, 1, 2, 0])).backward()
    g1 = flat.grad.clone()
    torch.nn.functional.cross_entropy(m(torch.randn(4, 8)), torch.tensor([0, 1, 2, 0])).backward()
    assert not torch.equal(flat.grad, g1)  # second backward accumulates


def test_optimizer_state_dict_roundtrip():
    m = _model()
    flat = FlatParams(m.parameters(), shadow_dtype=None)
    o = popt.Adam(flat, lr=1e-3)
    torch.nn.functional.cross_entropy(m(torch.randn(4, 8)), torch.tensor([0, 1, 2, 0])).backward()
    o.step()
    sd = o.state_dict()
    o2 = popt.Adam(flat, lr=5.0)
    o2.load_state_dict(sd)
    assert o2.lr == 1e-3 and torch.equal(o2.m1, o.m1) and o2.steps == 1

