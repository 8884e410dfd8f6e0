"""CPU checks of the transparent managed mode's dispatch plumbing
(open-gpu-kernel-modules_amd/managed.py): every aten op of a training step is
intercepted (forward, autograd backward, optimizer), and multi-tensor
``_foreach_*`` ops are split into slices that fit the arena with identical
results. The residency side (op holds) is covered on the fake backend in
tests/test_allocator.py and end to end on the GPU in test_managed_mode_gpu.py."""
from __future__ import annotations

import torch
from torch.utils._python_dispatch import TorchDispatchMode

import ogkm


def _model():
    torch.manual_seed(0)
    layer = torch.nn.TransformerEncoderLayer(64, 4, 128, dropout=0.0, batch_first=True)
    return torch.nn.TransformerEncoder(layer, 2, enable_nested_tensor=False)


def _step(model, x, foreach):
    opt = torch.optim.SGD(model.parameters(), lr=1e-2, foreach=foreach)
    y = model(x)
    y.pow(2).mean().backward()
    opt.step()
    return [p.detach().clone() for p in model.parameters()]


def test_mode_intercepts_forward_backward_and_optimizer():
    x = torch.randn(2, 8, 64)
    ref = _step(_model(), x, foreach=True)
    m = ogkm.managed(lookahead_bytes=0)
    seen = []
    orig = type(m).__torch_dispatch__

    def spy(self, func, types, args=(), kwargs=None):
        seen.append(func.__name__)
        return orig(self, func, types, args, kwargs)

    type(m).__torch_dispatch__ = spy
    try:
        TorchDispatchMode.__enter__(m)
        try:
            out = _step(_model(), x, foreach=True)
        finally:
            TorchDispatchMode.__exit__(m, None, None, None)
    finally:
        type(m).__torch_dispatch__ = orig
    assert all(torch.equal(a, b) for a, b in zip(ref, out))
    names = set(seen)
    assert any(n.startswith("mm") or n.startswith("addmm") for n in names), names  # forward GEMMs
    assert any("backward" in n for n in names) or "threshold_backward" in names or len(seen) > 100
    assert any(n.startswith("_foreach_add") for n in names), names  # the optimizer step


def test_foreach_ops_are_split_to_fit_the_arena():
    x = torch.randn(2, 8, 64)
    ref = _step(_model(), x, foreach=True)
    m = ogkm.managed(lookahead_bytes=0)
    m._arena_bytes = lambda: 64 << 10  # pretend a 64 KB arena: every foreach op is split
    calls = []
    orig = m._split_foreach

    def count(func, args, kwargs):
        r = orig(func, args, kwargs)
        calls.append(func.__name__)
        return r

    m._split_foreach = count
    TorchDispatchMode.__enter__(m)
    try:
        out = _step(_model(), x, foreach=True)
    finally:
        TorchDispatchMode.__exit__(m, None, None, None)
    assert calls, "no foreach op seen"
    assert all(torch.equal(a, b) for a, b in zip(ref, out))
