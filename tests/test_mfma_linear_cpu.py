"""The bf16 MFMA Linear chain (ops/mfma_linear.py) on the CPU: its autograd Function through the
kernels' reference ops against plain autograd, and which module structures the engine's kernel
injection takes (the GPU runs of the same code: tests/test_gpu_engine.py)."""
import copy

import pytest
import torch
import torch.nn as nn

from distributed_gpu_test_amd.models.synthetic_mlp import SyntheticMLP
from distributed_gpu_test_amd.ops import linear as lin_ops
from distributed_gpu_test_amd.ops.mfma_linear import (MfmaSequential, MfmaSyntheticMLP, _MfmaChainFn, chain_layout,
                                                       inject_mfma_linear)


def _wb(linears):
    out = []
    for l in linears:
        out += [l.weight, l.bias]
    return out


@pytest.mark.parametrize("head,need_dx", [(True, False), (False, False), (True, True)])
def test_chain_function_matches_autograd(head, need_dx):
    torch.manual_seed(0)
    layers = [nn.Linear(256, 256), nn.Linear(256, 128)] + ([nn.Linear(128, 2)] if head else [])
    relus = (True, True, False) if head else (True, False)
    mods = [l.to(torch.bfloat16) for l in layers]
    ref = [copy.deepcopy(l) for l in mods]
    x0 = torch.randn(128, 256).to(torch.bfloat16)
    x1, x2 = x0.clone().requires_grad_(need_dx), x0.clone().requires_grad_(need_dx)
    out = _MfmaChainFn.apply(x1, relus, head, False, *_wb(mods))
    h = x2
    for l, r in zip(ref, relus):
        h = l(h)
        h = torch.relu(h) if r else h
    dout = torch.randn_like(out)
    out.backward(dout)
    h.backward(dout)
    torch.testing.assert_close(out.float(), h.float(), rtol=2e-2, atol=2e-2)
    for a, b in zip(mods, ref):
        for p, q in ((a.weight, b.weight), (a.bias, b.bias)):
            scale = float(q.grad.float().abs().max()) + 1e-6
            torch.testing.assert_close(p.grad.float() / scale, q.grad.float() / scale, rtol=0, atol=2e-2)
    if need_dx:
        scale = float(x2.grad.float().abs().max())
        torch.testing.assert_close(x1.grad.float() / scale, x2.grad.float() / scale, rtol=0, atol=2e-2)


def test_injection_structures_and_keys():
    m = SyntheticMLP(256, 2).to(torch.bfloat16)
    keys = list(m.state_dict())
    assert inject_mfma_linear(m, grad_in_place=True) == 3 and type(m) is MfmaSyntheticMLP
    assert list(m.state_dict()) == keys
    seq = nn.Sequential(nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 1)).to(torch.bfloat16)
    assert inject_mfma_linear(seq) == 2 and type(seq) is MfmaSequential
    wrapper = nn.Module()
    wrapper.body = nn.Sequential(nn.Linear(128, 128), nn.ReLU(), nn.Linear(128, 128)).to(torch.bfloat16)
    assert inject_mfma_linear(wrapper) == 2 and type(wrapper.body) is MfmaSequential
    small = nn.Sequential(nn.Linear(20, 64), nn.ReLU(), nn.Linear(64, 1)).to(torch.bfloat16)
    before = dict(lin_ops.FALLBACKS)
    assert inject_mfma_linear(small) == 0 and type(small) is nn.Sequential
    assert sum(lin_ops.FALLBACKS.values()) > sum(before.values())  # counted, not silent
    assert chain_layout([nn.Linear(256, 256), nn.Linear(256, 3)], [True, False]) is True
    assert chain_layout([nn.Linear(256, 256), nn.Linear(256, 3)], [True, True]) is None  # ReLU after a head
    assert chain_layout([nn.Linear(256, 256), nn.Linear(128, 1)], [True, False]) is None  # shape mismatch


def test_injected_module_on_cpu_falls_back_and_counts():
    """A CPU input never reaches the kernels: the module's own forward runs, and it is counted."""
    torch.manual_seed(1)
    m = SyntheticMLP(256, 2).to(torch.bfloat16)
    ref = copy.deepcopy(m)
    inject_mfma_linear(m)
    x = torch.randn(128, 256).to(torch.bfloat16)
    n0 = sum(lin_ops.FALLBACKS.values())
    assert torch.equal(m(x), ref(x))
    assert sum(lin_ops.FALLBACKS.values()) == n0 + 1


def test_first_write_stores_once_per_backward():
    """engine_backward(grads_zero=True): the first write of a gradient view in that backward may
    store (the bucket is zero), every later write of the same view must add -- a module called
    twice before one backward writes its gradients twice; nested / later backwards start afresh."""
    import torch
    from distributed_gpu_test_amd.ops.linear import _first_write, engine_backward
    buf = torch.zeros(64)
    a, b = buf[:32], buf[32:]
    assert not _first_write(a)  # outside an engine backward: always accumulate
    with engine_backward(grads_zero=True):
        assert _first_write(a) and _first_write(b)
        assert not _first_write(a) and not _first_write(b)
    with engine_backward(grads_zero=True):
        assert _first_write(a)  # a new backward
    with engine_backward(grads_zero=False):
        assert not _first_write(a)  # the bucket already holds gradients (accumulation step)
